"""CLI: run a DeepSpeed autotuning search against a master with a local search runner."""
import argparse
import json
import os
import sys

import yaml

from determined_clone_amd import searcher
from determined_clone_amd.pytorch.dsat import _defaults
from determined_clone_amd.pytorch.dsat._search import DSATSearchMethod


def parse_args(argv=None) -> argparse.Namespace:
    d = _defaults.ARG_DEFAULTS
    p = argparse.ArgumentParser(prog="dsat", description="DeepSpeed autotune (MI355X native engine)")
    p.add_argument("search_method", choices=_defaults.SEARCH_METHODS)
    p.add_argument("config_path")
    p.add_argument("model_dir")
    p.add_argument("-mt", "--max-trials", type=int, default=d["max_trials"])
    p.add_argument("-mct", "--max-concurrent-trials", type=int, default=d["max_concurrent_trials"])
    p.add_argument("-m", "--metric", default=d["metric"],
                   choices=_defaults.SMALLER_IS_BETTER_METRICS + _defaults.LARGER_IS_BETTER_METRICS)
    p.add_argument("-z", "--zero-stages", type=int, nargs="+", default=d["zero_stages"], choices=[0, 1, 2, 3])
    p.add_argument("--start-profile-step", type=int, default=d["start_profile_step"])
    p.add_argument("--end-profile-step", type=int, default=d["end_profile_step"])
    p.add_argument("--max-mbs", type=int, default=d["max_mbs"])
    p.add_argument("-r", "--random-seed", type=int, default=d["random_seed"])
    p.add_argument("--searcher-dir", default="dsat_state")
    p.add_argument("--master", default=os.environ.get("DET_MASTER", "http://127.0.0.1:8080"))
    return p.parse_args(argv)


def build_method(args: argparse.Namespace, cfg: dict) -> DSATSearchMethod:
    hp = {k: (v["val"] if isinstance(v, dict) and v.get("type") == "const" else v)
          for k, v in (cfg.get("hyperparameters") or {}).items()}
    return DSATSearchMethod(hp, args.search_method, args.metric, tuple(args.zero_stages),
                            args.max_trials, args.max_concurrent_trials, args.start_profile_step,
                            args.end_profile_step, args.max_mbs, args.random_seed)


def main(argv=None, session=None) -> int:
    args = parse_args(argv)
    cfg = yaml.safe_load(open(args.config_path))
    cfg["searcher"] = {"name": "custom", "metric": args.metric, "unit": "batches",
                       "smaller_is_better": args.metric in _defaults.SMALLER_IS_BETTER_METRICS}
    method = build_method(args, cfg)
    if session is None:
        from determined_clone_amd.common.api import Session

        session = Session(args.master)
        session.token = session.post("/api/v1/auth/login", {"username": os.environ.get("DET_USER", "admin"),
                                                            "password": os.environ.get("DET_PASS", "")})["token"]
    runner = searcher.LocalSearchRunner(method, searcher_dir=args.searcher_dir, session=session)
    eid = runner.run(cfg, model_dir=args.model_dir)
    print(json.dumps({"experiment_id": eid, "best": method.best(), "trials": method.results()}))
    return 0


if __name__ == "__main__":
    sys.exit(main())
