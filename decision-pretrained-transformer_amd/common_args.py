"""argparse flag groups — same flags, types and defaults as the reference common_args.py:2-59."""

# (flag, type, default, help); flags with type=None are store_true switches.
DATASET_ARGS = [
    ("--envs", int, 100000, "Envs"),
    ("--envs_eval", int, 100, "Eval Envs"),
    ("--hists", int, 1, "Histories"),
    ("--samples", int, 1, "Samples"),
    ("--H", int, 100, "Context horizon"),
    ("--dim", int, 10, "Dimension"),
    ("--lin_d", int, 2, "Linear feature dimension"),
    ("--var", float, 0.0, "Bandit arm variance"),
    ("--cov", float, 0.0, "Coverage of optimal arm"),
    ("--env", str, None, "Environment"),          # required
    ("--env_id_start", int, -1, "Start index of envs to sample"),
    ("--env_id_end", int, -1, "End index of envs to sample"),
]
MODEL_ARGS = [
    ("--embd", int, 32, "Embedding size"),
    ("--head", int, 1, "Number of heads"),
    ("--layer", int, 3, "Number of layers"),
    ("--lr", float, 1e-3, "Learning Rate"),
    ("--dropout", float, 0, "Dropout"),
    ("--shuffle", None, False, None),
]
TRAIN_ARGS = [("--num_epochs", int, 1000, "Number of epochs")]
EVAL_ARGS = [
    ("--epoch", int, -1, "Epoch to evaluate"),
    ("--test_cov", float, -1.0, "Test coverage (for bandit)"),
    ("--hor", int, -1, "Episode horizon (for mdp)"),
    ("--n_eval", int, 100, "Number of eval trajectories"),
    ("--save_video", None, False, None),
]
REQUIRED = {"--env"}


def _add(parser, table):
    for flag, typ, default, helptext in table:
        if typ is None:
            parser.add_argument(flag, default=default, action="store_true")
        elif flag in REQUIRED:
            parser.add_argument(flag, type=typ, required=True, help=helptext)
        else:
            parser.add_argument(flag, type=typ, required=False, default=default, help=helptext)


def add_dataset_args(parser):
    _add(parser, DATASET_ARGS)


def add_model_args(parser):
    _add(parser, MODEL_ARGS)


def add_train_args(parser):
    _add(parser, TRAIN_ARGS)


def add_eval_args(parser):
    _add(parser, EVAL_ARGS)
