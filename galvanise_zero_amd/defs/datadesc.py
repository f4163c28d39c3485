"""Data records of the hot path: Sample (reference src/ggpzero/defs/datadesc.py:8-38, the dict
layout sampleToDict emits, supervisor_impl.cpp:75-118), GenerationSamples (datadesc.py:40-52) and
GenerationDescription (datadesc.py:55-95)."""
import attr

from ..util.attrutil import register_attrs

_WIRE = "ggpzero.defs.datadesc"     # module name in the reference's JSON class tags


@register_attrs(_WIRE)
@attr.s
class Sample(object):
    state = attr.ib(default=attr.Factory(list))
    prev_states = attr.ib(default=attr.Factory(list))
    policies = attr.ib(default=attr.Factory(list))
    final_score = attr.ib(default=attr.Factory(list))
    depth = attr.ib(default=0)
    game_length = attr.ib(default=0)
    match_identifier = attr.ib(default="")
    has_resigned = attr.ib(default=False)
    resign_false_positive = attr.ib(default=False)
    starting_sample_depth = attr.ib(default=0)
    resultant_puct_score = attr.ib(default=attr.Factory(list))
    resultant_puct_visits = attr.ib(default=0)


@register_attrs(_WIRE)
@attr.s
class GenerationSamples(object):
    """datadesc.py:40-52: one gendata_<game>_<step>.json.gz file."""
    game = attr.ib(default="game")
    date_created = attr.ib(default="2018-01-24 22:28")
    with_generation = attr.ib(default="v6_123")
    num_samples = attr.ib(default=1024)
    samples = attr.ib(default=attr.Factory(list))


@register_attrs(_WIRE)
@attr.s
class GenerationDescription(object):
    game = attr.ib(default="breakthrough")
    name = attr.ib(default="v6_123")
    date_created = attr.ib(default="2018-01-24 22:28")
    channel_last = attr.ib(default=False)
    multiple_policy_heads = attr.ib(default=False)
    num_previous_states = attr.ib(default=0)
    transformer_description = attr.ib(default=None)
    draw_head = attr.ib(default=False)
    trained_losses = attr.ib(default="not set")
    trained_validation_losses = attr.ib(default="not set")
    trained_policy_accuracy = attr.ib(default="not set")
    trained_value_accuracy = attr.ib(default="not set")
