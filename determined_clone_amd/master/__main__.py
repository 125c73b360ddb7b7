"""``python -m determined_clone_amd.master`` — run the master (reference: determined-master)."""
import argparse
import logging
import os
import signal
import threading

import yaml

from determined_clone_amd.master import Master, MasterServer


def main() -> None:
    ap = argparse.ArgumentParser("det-clone-master")
    ap.add_argument("--config-file", default=None, help="master.yaml")
    ap.add_argument("--host", default="127.0.0.1")
    ap.add_argument("--port", type=int, default=8080)
    ap.add_argument("--db", default=os.path.join(os.path.expanduser("~"), ".det-clone-master.db"))
    ap.add_argument("--scheduler", default=None, choices=[None, "priority", "fair_share", "round_robin"])
    ap.add_argument("--fit", default=None, choices=[None, "best", "worst"])
    ap.add_argument("--checkpoint-dir", default=None)
    ap.add_argument("--authz", default=None, choices=[None, "basic", "rbac"],
                    help="security.authz.type: basic (admin-only cluster administration) or rbac")
    args = ap.parse_args()
    cfg = {}
    if args.config_file:
        with open(args.config_file) as f:
            cfg = yaml.safe_load(f) or {}
    sched = (cfg.get("resource_manager") or {}).get("scheduler") or {}
    logging.basicConfig(level=logging.INFO, format="%(asctime)s %(levelname)s %(name)s: %(message)s")
    cs = cfg.get("checkpoint_storage")
    if args.checkpoint_dir:
        cs = {"type": "shared_fs", "host_path": args.checkpoint_dir}
    m = Master(args.db, scheduler=args.scheduler or sched.get("type", "priority"),
               fit=args.fit or sched.get("fitting_policy", "best"),
               preemption=bool(sched.get("preemption", True)), checkpoint_storage=cs,
               cluster_name=cfg.get("cluster_name", "default"),
               authz=args.authz or ((cfg.get("security") or {}).get("authz") or {}).get("type", "basic"),
               resource_manager=cfg.get("resource_manager"), resource_pools=cfg.get("resource_pools"),
               logging_config=cfg.get("logging"), webhooks_config=cfg.get("webhooks"))
    m.sso_providers = [{"name": str(p["name"]), "sso_url": str(p["sso_url"])}
                       for p in cfg.get("sso_providers") or []]
    srv = MasterServer(m, cfg.get("host", args.host), int(cfg.get("port", args.port)),
                       tls=(cfg.get("security") or {}).get("tls"))
    if cfg.get("external_url"):  # the address tasks, agents and provisioned instances dial
        m.master_url = str(cfg["external_url"]).rstrip("/")
    srv.start()
    logging.info(f"master listening on {m.master_url}")
    stop = threading.Event()
    signal.signal(signal.SIGTERM, lambda *a: stop.set())
    try:
        stop.wait()
    except KeyboardInterrupt:
        pass
    srv.stop()


if __name__ == "__main__":
    main()
