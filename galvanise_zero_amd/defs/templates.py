"""Config templates (reference src/ggpzero/defs/templates.py:7-129): generation description,
network size hints, base PUCT config and the self-play template the BASELINE "template" mode uses."""
from datetime import datetime

from . import confs, datadesc


def default_generation_desc(game, name="default", **kwds):
    desc = datadesc.GenerationDescription(game)
    desc.name = name
    desc.date_created = datetime.now().strftime("%Y/%m/%d %H:%M")
    desc.channel_last = False
    desc.multiple_policy_heads = True
    desc.num_previous_states = 0
    for k, v in kwds.items():
        setattr(desc, k, v)
    return desc


_SIZES = {"small": (64, 5, 256), "medium": (96, 5, 512), "large": (96, 10, 512)}


def nn_model_config_template(game, network_size_hint, transformer, features=False):
    conf = confs.NNModelConfig()
    conf.role_count = transformer.role_count
    conf.input_rows = transformer.num_rows
    conf.input_columns = transformer.num_cols
    conf.input_channels = transformer.num_channels
    conf.policy_dist_count = list(transformer.policy_dist_count)
    conf.cnn_kernel_size = 3
    conf.dropout_rate_policy = 0.25
    conf.dropout_rate_value = 0.5
    if network_size_hint not in _SIZES:
        raise ValueError("network_size_hint %s, not recognised" % network_size_hint)
    conf.cnn_filter_size, conf.residual_layers, conf.value_hidden_size = _SIZES[network_size_hint]
    conf.leaky_relu = False
    conf.resnet_v2 = conf.squeeze_excite_layers = conf.global_pooling_value = bool(features)
    return conf


def base_puct_config(**kwds):
    config = confs.PUCTEvaluatorConfig(verbose=False, backup_finalised=False, batch_size=1,
                                       dirichlet_noise_pct=-1, puct_constant=0.85, puct_constant_root=0.85,
                                       fpu_prior_discount=0.25, fpu_prior_discount_root=0.25,
                                       choose="choose_temperature", temperature=1.0, depth_temperature_max=5.0,
                                       depth_temperature_start=2, depth_temperature_increment=0.2,
                                       depth_temperature_stop=6, random_scale=0.95, think_time=-1,
                                       max_dump_depth=0, top_visits_best_guess_converge_ratio=0.85,
                                       converged_visits=1, evaluation_multiplier_to_convergence=2.0)
    for k, v in kwds.items():
        setattr(config, k, v)
    return config


def selfplay_config_template():
    conf = confs.SelfPlayConfig()
    conf.oscillate_sampling_pct = 0.25
    conf.temperature_for_policy = 1.0
    conf.puct_config = base_puct_config(dirichlet_noise_pct=0.25)
    conf.evals_per_move = 100
    conf.resign0_score_probability = 0.1
    conf.resign0_pct = 0.99
    conf.resign1_score_probability = 0.025
    conf.resign1_pct = 0.95
    conf.run_to_end_pct = 0.01
    conf.run_to_end_evals = 32
    conf.run_to_end_puct_config = base_puct_config(dirichlet_noise_pct=0.15, random_scale=0.75)
    conf.run_to_end_early_score = 0.01
    conf.run_to_end_minimum_game_depth = 30
    conf.abort_max_length = -1
    return conf


def literal_selfplay_config(evals_per_move):
    """BASELINE "literal" mode: every move is a sampled move of exactly
    evals_per_move NN evaluations: no oscillation, convergence multiplier 1, resignation off."""
    conf = selfplay_config_template()
    conf.evals_per_move = evals_per_move
    conf.oscillate_sampling_pct = -1
    conf.puct_config.evaluation_multiplier_to_convergence = 1.0
    conf.resign0_pct = 1.0
    conf.resign1_pct = 1.0
    return conf
