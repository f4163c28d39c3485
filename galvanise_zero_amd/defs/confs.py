"""Config records consumed by the self-play hot path.

Field names and defaults restate reference src/ggpzero/defs/confs.py:9-151 (PUCTEvaluatorConfig,
PUCTPlayerConfig, SelfPlayConfig, NNModelConfig); tests/golden/configs.json (generated from the
reference by tests/golden/make_config_golden.py) pins them.
"""
import attr


def _f(default):
    return attr.ib(default=default)


@attr.s
class PUCTEvaluatorConfig(object):
    verbose = _f(False)
    puct_constant = _f(0.85)
    puct_constant_root = _f(2.5)
    dirichlet_noise_pct = _f(0.25)
    noise_policy_squash_pct = _f(-1)
    noise_policy_squash_prob = _f(0.05)
    choose = _f("choose_top_visits")
    max_dump_depth = _f(2)
    random_scale = _f(0.5)
    temperature = _f(1.0)
    depth_temperature_start = _f(5)
    depth_temperature_increment = _f(0.5)
    depth_temperature_stop = _f(10)
    depth_temperature_max = _f(5.0)
    fpu_prior_discount = _f(0.25)
    fpu_prior_discount_root = _f(0.25)
    think_time = _f(10.0)
    converged_visits = _f(5000)
    top_visits_best_guess_converge_ratio = _f(0.8)
    evaluation_multiplier_to_convergence = _f(1.0)
    batch_size = _f(32)
    use_legals_count_draw = _f(-1)
    backup_finalised = _f(False)
    lookup_transpositions = _f(False)


@attr.s
class PUCTPlayerConfig(object):
    name = _f("Player")
    verbose = _f(False)
    playouts_per_iteration = _f(800)
    playouts_per_iteration_noop = _f(1)
    generation = _f("latest")
    evaluator_config = attr.ib(factory=PUCTEvaluatorConfig)


@attr.s
class SelfPlayConfig(object):
    oscillate_sampling_pct = _f(0.25)
    temperature_for_policy = _f(1.0)
    puct_config = attr.ib(factory=PUCTEvaluatorConfig)
    evals_per_move = _f(800)
    resign0_score_probability = _f(0.9)
    resign0_pct = _f(0.5)
    resign1_score_probability = _f(0.975)
    resign1_pct = _f(0.1)
    run_to_end_pct = _f(0.2)
    run_to_end_evals = _f(42)
    run_to_end_puct_config = attr.ib(factory=PUCTEvaluatorConfig)
    run_to_end_early_score = _f(0.01)
    run_to_end_minimum_game_depth = _f(30)
    abort_max_length = _f(-1)


@attr.s
class NNModelConfig(object):
    role_count = _f(2)
    input_rows = _f(8)
    input_columns = _f(8)
    input_channels = _f(8)
    residual_layers = _f(8)
    cnn_filter_size = _f(64)
    cnn_kernel_size = _f(3)
    value_hidden_size = _f(256)
    policy_dist_count = attr.ib(factory=list)
    dropout_rate_policy = _f(0.333)
    dropout_rate_value = _f(0.5)
    leaky_relu = _f(False)
    squeeze_excite_layers = _f(False)
    resnet_v2 = _f(False)
    global_pooling_value = _f(False)
    concat_all_layers = _f(False)
