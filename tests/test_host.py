"""Host-side drop-in surface on CPU: filenames and CLI flags equal the reference's
(tests/golden/host_surface.json, recorded from the reference's utils.py / common_args.py)."""
import argparse
import json
import os

from conftest import GOLDEN


def surface():
    return json.load(open(os.path.join(GOLDEN, "host_surface.json")))


def test_filenames_match_reference():
    import utils
    for fn, args, expected in surface()["filenames"]:
        assert getattr(utils, fn)(*args) == expected, (fn, args)


def test_flag_defaults_match_reference():
    import common_args
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_train_args(p)
    common_args.add_eval_args(p)
    assert vars(p.parse_args(["--env", "bandit"])) == surface()["defaults"]


def test_run_scripts_parse():
    """The reference recipes' collect / eval command lines parse with our CLIs (run_bandit.sh:2,8)."""
    import common_args
    collect = "--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --envs_eval 200".split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    a = vars(p.parse_args(collect))
    assert a["H"] == 500 and a["envs_eval"] == 200
    ev = ("--env bandit --envs 100000 --H 500 --dim 5 --var 0.3 --cov 0.0 --lr 0.0001 --layer 4 --head 4 "
          "--shuffle --epoch 50 --n_eval 200 --seed 1").split()
    p = argparse.ArgumentParser()
    common_args.add_dataset_args(p)
    common_args.add_model_args(p)
    common_args.add_eval_args(p)
    p.add_argument("--seed", type=int, default=0)
    a = vars(p.parse_args(ev))
    assert a["shuffle"] is True and a["layer"] == 4 and a["epoch"] == 50
