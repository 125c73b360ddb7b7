"""``det deploy gke``: a GKE cluster with a CPU node pool for the master and an accelerator
node pool for tasks, then the Kubernetes installation of ``deploy/kubernetes.py`` (reference:
`deploy/gke/cli.py`, which drives ``gcloud container clusters create`` / ``node-pools create``
and then ``helm install`` of the Determined chart).

Every external step is a ``gcloud`` / ``kubectl`` invocation built by ``plan()``, so ``--dry-run``
prints the exact commands and tests can check them without a cloud. Task pods request the
node pool's accelerator resource; for AMD Instinct node pools that is ``amd.com/gpu`` (the
default), for other accelerators pass ``--slot-resource``."""
import subprocess
from typing import Any, Callable, Dict, List, Optional

from determined_clone_amd.deploy import kubernetes as k8s


def _base(args: Any) -> List[str]:
    return ["--region", args.region] if getattr(args, "region", None) else ["--zone", args.zone]


def plan(args: Any) -> List[List[str]]:
    cid = args.cluster_id
    loc = _base(args)
    cmds = [
        ["gcloud", "container", "clusters", "create", cid, *loc, "--num-nodes", "1",
         "--machine-type", args.master_machine_type, "--enable-ip-alias", "--quiet",
         "--labels", f"determined-clone-amd-cluster={cid}"],
        ["gcloud", "container", "node-pools", "create", args.gpu_node_pool_name, "--cluster", cid, *loc,
         "--machine-type", args.agent_machine_type, "--num-nodes", "0",
         "--enable-autoscaling", "--min-nodes", "0", "--max-nodes", str(args.max_gpu_nodes),
         "--node-labels", "determined.ai/resource_pool=default", "--quiet"]
        + (["--accelerator", f"type={args.gpu_type},count={args.gpus_per_node}"] if args.gpu_type else []),
        ["gcloud", "container", "clusters", "get-credentials", cid, *loc],
    ]
    if not getattr(args, "no_managed_bucket", False):
        bucket = args.gcs_bucket_name or f"det-{cid}-checkpoints"
        cmds.insert(0, ["gcloud", "storage", "buckets", "create", f"gs://{bucket}", "--location",
                        (args.region or args.zone.rsplit("-", 1)[0])])
    return cmds


def install_values(args: Any) -> Dict[str, Any]:
    v: Dict[str, Any] = {"namespace": args.namespace, "image": args.image, "release": "det",
                         "slot_resource": args.slot_resource, "max_slots_per_pod": args.gpus_per_node,
                         "service_type": "LoadBalancer"}
    if not getattr(args, "no_managed_bucket", False):
        v["checkpoint_storage"] = {"type": "gcs", "bucket": args.gcs_bucket_name or f"det-{args.cluster_id}-checkpoints"}
    elif args.gcs_bucket_name:
        v["checkpoint_storage"] = {"type": "gcs", "bucket": args.gcs_bucket_name}
    return v


def _run(cmd: List[str], runner: Callable[..., Any]) -> None:
    try:
        runner(cmd, check=True)
    except FileNotFoundError:
        raise RuntimeError(f"{cmd[0]} not found on PATH (use --dry-run to print the commands)")


def up(args: Any, log: Callable[[str], None] = print, runner: Callable[..., Any] = subprocess.run,
       kubectl_bin: str = "kubectl") -> Optional[Dict[str, Any]]:
    cmds = plan(args)
    if getattr(args, "dry_run", False):
        for c in cmds:
            log(" ".join(c))
        log(f"kubectl apply -f - <<< (det deploy k8s render, namespace {args.namespace})")
        return None
    for c in cmds:
        log("+ " + " ".join(c))
        _run(c, runner)
    return k8s.up(install_values(args), kubectl_bin=kubectl_bin)


def down(args: Any, log: Callable[[str], None] = print, runner: Callable[..., Any] = subprocess.run) -> None:
    cmd = ["gcloud", "container", "clusters", "delete", args.cluster_id, *_base(args), "--quiet"]
    log("+ " + " ".join(cmd))
    _run(cmd, runner)
    log("cluster deleted (the checkpoint bucket is kept)")
