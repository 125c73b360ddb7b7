"""CLI: run a DeepSpeed autotuning search against a master with a local search runner
(reference: `harness/determined/pytorch/dsat/__main__.py`, `_run_dsat.py`).

``python -m determined_clone_amd.pytorch.dsat {binary,random,asha,_test} config.yaml model_dir``
submits a custom-searcher experiment whose trials profile DeepSpeed configurations, prints the best
one as JSON, and with ``--run-full-experiment`` then submits the original experiment with that
configuration merged into its ``overwrite_deepspeed_args``."""
import argparse
import base64
import copy
import json
import os
import shutil
import sys
import tempfile

import yaml

from determined_clone_amd import searcher
from determined_clone_amd.pytorch.dsat import _defaults, _utils
from determined_clone_amd.pytorch.dsat._asha import ASHADSATSearchMethod
from determined_clone_amd.pytorch.dsat._search import DSATSearchMethod


def parse_args(argv=None) -> argparse.Namespace:
    d = _defaults.ARG_DEFAULTS
    p = argparse.ArgumentParser(prog="dsat", description="DeepSpeed autotune (MI355X native engine)",
                                formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    p.add_argument("search_method", choices=_defaults.SEARCH_METHODS)
    p.add_argument("config_path", help="experiment config (.yaml)")
    p.add_argument("model_dir", help="directory with the model definition")
    p.add_argument("-i", "--include", nargs="+", default=[],
                   help="additional files / directories copied into the model directory")
    p.add_argument("-mt", "--max-trials", type=int, default=d["max_trials"])
    p.add_argument("-ms", "--max-slots", type=int, default=None,
                   help="cap on slots in use at once (limits concurrent trials by slots_per_trial)")
    p.add_argument("-mct", "--max-concurrent-trials", type=int, default=d["max_concurrent_trials"])
    p.add_argument("-m", "--metric", default=d["metric"],
                   choices=_defaults.SMALLER_IS_BETTER_METRICS + _defaults.LARGER_IS_BETTER_METRICS)
    p.add_argument("--run-full-experiment", action="store_true",
                   help="submit the full-length experiment with the best configuration afterwards")
    p.add_argument("-z", "--zero-stages", type=int, nargs="+", default=d["zero_stages"], choices=[0, 1, 2, 3])
    p.add_argument("--start-profile-step", type=int, default=d["start_profile_step"])
    p.add_argument("--end-profile-step", type=int, default=d["end_profile_step"])
    p.add_argument("--max-mbs", type=int, default=d["max_mbs"])
    p.add_argument("-r", "--random-seed", type=int, default=d["random_seed"])
    # random
    p.add_argument("--trials-per-random-config", type=int, default=d["trials_per_random_config"])
    p.add_argument("--early-stopping", type=int, default=None,
                   help="random: stop after this many completed trials without a new best")
    # binary / asha
    p.add_argument("--search-range-factor", type=float, default=d["search_range_factor"])
    # asha
    p.add_argument("--divisor", type=int, default=d["divisor"], help="ASHA eta")
    p.add_argument("--min-binary-search-trials", type=int, default=d["min_binary_search_trials"])
    p.add_argument("--max-rungs", type=int, default=d["max_rungs"])
    p.add_argument("--asha-early-stopping", type=int, default=d["asha_early_stopping"], help="ASHA s")
    p.add_argument("--searcher-dir", default="dsat_state")
    p.add_argument("--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    return p.parse_args(argv)


def _const_hparams(cfg: dict) -> dict:
    return {k: (v["val"] if isinstance(v, dict) and v.get("type") == "const" else v)
            for k, v in (cfg.get("hyperparameters") or {}).items()}


def build_method(args: argparse.Namespace, cfg: dict) -> searcher.SearchMethod:
    hp = _const_hparams(cfg)
    slots = int((cfg.get("resources") or {}).get("slots_per_trial", 1) or 1)
    concurrent = args.max_concurrent_trials
    if args.max_slots:
        concurrent = max(1, min(concurrent, args.max_slots // slots))
    if args.search_method == "asha":
        return ASHADSATSearchMethod(
            hp, args.metric, tuple(args.zero_stages), args.max_trials, concurrent,
            args.start_profile_step, args.end_profile_step, args.max_mbs, args.random_seed,
            divisor=args.divisor, min_binary_search_trials=args.min_binary_search_trials,
            max_rungs=args.max_rungs, asha_early_stopping=args.asha_early_stopping,
            search_range_factor=args.search_range_factor, slots_per_trial=slots)
    return DSATSearchMethod(hp, args.search_method, args.metric, tuple(args.zero_stages),
                            args.max_trials, concurrent, args.start_profile_step,
                            args.end_profile_step, args.max_mbs, args.random_seed,
                            early_stopping=args.early_stopping)


def full_experiment_config(cfg: dict, best: dict) -> dict:
    """The submitted experiment with the winning DeepSpeed settings merged into its
    ``overwrite_deepspeed_args`` hyperparameter (searcher and length unchanged)."""
    out = copy.deepcopy(cfg)
    zero = dict(best.get("zero_optimization") or {"stage": best["zero_stage"]})
    ow = {"train_micro_batch_size_per_gpu": best["train_micro_batch_size_per_gpu"],
          "zero_optimization": zero}
    hps = out.setdefault("hyperparameters", {})
    prev = hps.get(_defaults.OVERWRITE_KEY) or {}
    if isinstance(prev, dict) and prev.get("type") == "const":
        prev = prev.get("val") or {}
    merged = _utils.merge_dicts(prev, ow)
    merged.pop("train_batch_size", None)
    hps[_defaults.OVERWRITE_KEY] = merged
    out["name"] = f"{cfg.get('name', 'experiment')} (dsat best)"
    return out


def main(argv=None, session=None) -> int:
    args = parse_args(argv)
    with open(args.config_path) as f:
        orig = yaml.safe_load(f)
    cfg = copy.deepcopy(orig)
    cfg["searcher"] = {"name": "custom", "metric": args.metric, "unit": "batches",
                       "smaller_is_better": _utils.smaller_is_better(args.metric)}
    method = build_method(args, cfg)
    if session is None:
        from determined_clone_amd.common.api import Session

        session = Session(args.master)
        session.token = session.post("/api/v1/auth/login", {"username": os.environ.get("DET_USER", "admin"),
                                                            "password": os.environ.get("DET_PASS", "")})["token"]
    model_dir = args.model_dir
    tmp = None
    if args.include:
        tmp = tempfile.mkdtemp(prefix="dsat-ctx-")
        model_dir = os.path.join(tmp, "ctx")
        shutil.copytree(args.model_dir, model_dir)
        for path in args.include:
            dst = os.path.join(model_dir, os.path.basename(os.path.normpath(path)))
            (shutil.copytree if os.path.isdir(path) else shutil.copy2)(path, dst)
    try:
        runner = searcher.LocalSearchRunner(method, searcher_dir=args.searcher_dir, session=session)
        eid = runner.run(cfg, model_dir=model_dir)
        best = method.best()
        out = {"experiment_id": eid, "best": best, "trials": method.results()}
        if args.run_full_experiment and best is not None:
            from determined_clone_amd.util import tar_directory

            body = {"config": full_experiment_config(orig, best),
                    "model_definition": base64.b64encode(tar_directory(model_dir)).decode()}
            out["full_experiment_id"] = int(session.post("/api/v1/experiments", body)["experiment"]["id"])
        print(json.dumps(out))
    finally:
        if tmp:
            shutil.rmtree(tmp, ignore_errors=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
