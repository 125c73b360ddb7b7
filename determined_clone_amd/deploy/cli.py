"""``det deploy {aws,gcp,gke,k8s}`` argument parsing (reference: `deploy/cli.py`,
`deploy/aws/cli.py`, `deploy/gcp/cli.py`, `deploy/gke/cli.py`)."""
import argparse
import json
import os
from typing import Any, Dict


def _aws(args: argparse.Namespace) -> None:
    from determined_clone_amd.deploy import aws

    if args.aws_cmd == "up":
        aws.up(args)
    elif args.aws_cmd == "down":
        if not args.yes and input(f"delete cluster {args.cluster_id}? [y/N] ").strip().lower() != "y":
            print("aborted")
            return
        aws.down(args)
    elif args.aws_cmd == "list":
        for s in aws.list_clusters(args):
            print(f"{s['name']}\t{s['status']}\t{s['outputs'].get('MasterAddress', '')}")
    elif args.aws_cmd == "print-template":
        print(json.dumps(aws.template(args.deployment_type), indent=2))


def _gcp(args: argparse.Namespace) -> None:
    from determined_clone_amd.deploy import gcp

    if args.gcp_cmd == "up":
        gcp.up(args)
    elif args.gcp_cmd == "down":
        if not args.yes and input(f"destroy cluster {args.cluster_id}? [y/N] ").strip().lower() != "y":
            print("aborted")
            return
        gcp.down(args)
    elif args.gcp_cmd == "list":
        for c in gcp.list_clusters(args):
            print(c)


def _gke(args: argparse.Namespace) -> None:
    from determined_clone_amd.deploy import gke

    if args.gke_cmd == "up":
        gke.up(args)
    else:
        gke.down(args)


def _k8s_values(args: argparse.Namespace) -> Dict[str, Any]:
    import yaml

    v: Dict[str, Any] = {}
    if args.values:
        with open(args.values) as f:
            v.update(yaml.safe_load(f) or {})
    for k in ("namespace", "image", "service_type", "storage_class", "max_slots_per_pod", "master_port"):
        x = getattr(args, k, None)
        if x is not None:
            v[k] = x
    return v


def _k8s(args: argparse.Namespace) -> None:
    from determined_clone_amd.deploy import kubernetes as k8s

    v = _k8s_values(args)
    if args.k8s_cmd == "render":
        print(k8s.to_yaml(k8s.render(v)), end="")
    elif args.k8s_cmd == "up":
        print(json.dumps(k8s.up(v, kubectl_bin=args.kubectl)))
    else:
        k8s.down(v, kubectl_bin=args.kubectl, delete_volumes=args.delete_volumes)


def register(sub: Any) -> None:
    """Add the cloud deployment commands to the ``det deploy`` subparsers."""
    # ---------------------------------------------------------------- aws
    a = sub.add_parser("aws", help="EC2 cluster as a CloudFormation stack").add_subparsers(dest="aws_cmd", required=True)
    for name in ("up", "down", "list", "print-template"):
        sp = a.add_parser(name)
        sp.set_defaults(func=_aws)
        sp.add_argument("--region", default=os.environ.get("AWS_REGION", "us-west-2"))
        sp.add_argument("--deployment-type", default="simple", choices=["simple", "vpc"])
        sp.add_argument("--endpoint-url", default=None, help=argparse.SUPPRESS)
        if name in ("up", "down"):
            sp.add_argument("--cluster-id", required=True)
            sp.add_argument("--no-wait", action="store_true")
            sp.add_argument("--yes", action="store_true")
        if name == "up":
            sp.add_argument("--keypair", required=True)
            sp.add_argument("--image-id", required=True, help="AMI with ROCm + this framework")
            sp.add_argument("--gpu-agent-instance-type", required=True)
            sp.add_argument("--master-instance-type", default="m7i.2xlarge")
            sp.add_argument("--inbound-cidr", default="0.0.0.0/0")
            sp.add_argument("--slots-per-instance", type=int, default=8)
            sp.add_argument("--min-dynamic-agents", type=int, default=0)
            sp.add_argument("--max-dynamic-agents", type=int, default=4)
            sp.add_argument("--max-idle-agent-period", default="10m")
            sp.add_argument("--scheduler-type", default="priority", choices=["priority", "fair_share", "round_robin"])
            sp.add_argument("--preemption-enabled", type=lambda s: s.lower() in ("1", "true", "yes"), default=True)
    # ---------------------------------------------------------------- gcp
    g = sub.add_parser("gcp", help="Compute Engine cluster through Terraform").add_subparsers(dest="gcp_cmd", required=True)
    for name in ("up", "down", "list"):
        sp = g.add_parser(name)
        sp.set_defaults(func=_gcp)
        sp.add_argument("--local-state-path", default=None)
        if name == "list":
            continue
        sp.add_argument("--cluster-id", required=True)
        sp.add_argument("--yes", action="store_true")
        if name == "up":
            sp.add_argument("--project-id", required=True)
            sp.add_argument("--region", default="us-central1")
            sp.add_argument("--zone", default=None)
            sp.add_argument("--environment-image", required=True, help="VM image with ROCm + this framework")
            sp.add_argument("--gpu-agent-instance-type", required=True)
            sp.add_argument("--gpu-type", default=None)
            sp.add_argument("--gpu-num", type=int, default=8)
            sp.add_argument("--master-instance-type", default="n2-standard-4")
            sp.add_argument("--inbound-cidr", default="0.0.0.0/0")
            sp.add_argument("--port", type=int, default=8080)
            sp.add_argument("--disk-size", type=int, default=500)
            sp.add_argument("--preemptible", action="store_true")
            sp.add_argument("--min-dynamic-agents", type=int, default=0)
            sp.add_argument("--max-dynamic-agents", type=int, default=4)
            sp.add_argument("--max-idle-agent-period", default="10m")
            sp.add_argument("--scheduler-type", default="priority")
            sp.add_argument("--tf-state-gcs-bucket-name", default=None)
            sp.add_argument("--dry-run", action="store_true")
    # ---------------------------------------------------------------- gke
    k = sub.add_parser("gke", help="GKE cluster + Kubernetes installation").add_subparsers(dest="gke_cmd", required=True)
    for name in ("up", "down"):
        sp = k.add_parser(name)
        sp.set_defaults(func=_gke)
        sp.add_argument("--cluster-id", required=True)
        sp.add_argument("--region", default=None)
        sp.add_argument("--zone", default="us-central1-a")
        if name == "up":
            sp.add_argument("--master-machine-type", default="n2-standard-4")
            sp.add_argument("--agent-machine-type", required=True)
            sp.add_argument("--gpu-type", default=None)
            sp.add_argument("--gpus-per-node", type=int, default=8)
            sp.add_argument("--max-gpu-nodes", type=int, default=4)
            sp.add_argument("--gpu-node-pool-name", default="accelerator-pool")
            sp.add_argument("--slot-resource", default="amd.com/gpu")
            sp.add_argument("--gcs-bucket-name", default=None)
            sp.add_argument("--no-managed-bucket", action="store_true")
            sp.add_argument("--namespace", default="determined")
            sp.add_argument("--image", default="determined-clone-amd:rocm7.2-gfx950")
            sp.add_argument("--dry-run", action="store_true")
    # ---------------------------------------------------------------- plain Kubernetes
    kk = sub.add_parser("k8s", help="install the master into an existing Kubernetes cluster").add_subparsers(
        dest="k8s_cmd", required=True)
    for name in ("render", "up", "down"):
        sp = kk.add_parser(name)
        sp.set_defaults(func=_k8s)
        sp.add_argument("--values", default=None, help="YAML file of deploy/kubernetes.py DEFAULTS overrides")
        sp.add_argument("--namespace", default=None)
        sp.add_argument("--image", default=None)
        sp.add_argument("--service-type", default=None, choices=[None, "ClusterIP", "NodePort", "LoadBalancer"])
        sp.add_argument("--storage-class", default=None)
        sp.add_argument("--max-slots-per-pod", type=int, default=None)
        sp.add_argument("--master-port", type=int, default=None)
        sp.add_argument("--kubectl", default="kubectl")
        sp.add_argument("--delete-volumes", action="store_true")
