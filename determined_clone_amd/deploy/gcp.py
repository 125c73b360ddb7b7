"""``det deploy gcp``: a cluster on Compute Engine through Terraform (reference:
`deploy/gcp/cli.py`, `deploy/gcp/gcp.py` and the HCL modules under `deploy/gcp/terraform/` --
network, firewall, service account, GCS bucket, static IP, master instance).

The configuration is generated as Terraform JSON (``main.tf.json``) from Python instead of shipping
HCL modules: one file, every value explicit, diffable. ``up`` runs ``terraform init`` + ``apply``
in the cluster's state directory, ``down`` runs ``destroy`` (after the master's provisioner-launched
agents are deleted), ``--dry-run`` writes the configuration and stops.

The master VM's startup script writes ``master.yaml`` (GCS checkpoints; a resource pool whose GCE
provisioner launches GPU agents under the cluster's service account) and starts the master;
credentials come from the metadata server, so nothing secret is written into the configuration."""
import json
import os
import subprocess
from typing import Any, Callable, Dict, List, Optional

import yaml

LABEL = "determined-clone-amd-cluster"


def _name(cluster_id: str, what: str) -> str:
    return f"det-{cluster_id}-{what}"[:62].rstrip("-")


def master_yaml(v: Dict[str, Any]) -> Dict[str, Any]:
    cid = v["cluster_id"]
    provider = {
        "type": "gcp", "project": v["project_id"], "zone": v["zone"],
        "boot_disk_source_image": v["environment_image"], "boot_disk_size": v["disk_size"],
        "instance_type": {"machine_type": v["gpu_agent_instance_type"], "gpu_type": v.get("gpu_type"),
                          "gpu_num": v["gpu_num"]},
        "slots_per_instance": v["gpu_num"],
        "min_instances": v["min_dynamic_agents"], "max_instances": v["max_dynamic_agents"],
        "max_idle_agent_period": v["max_idle_agent_period"],
        "max_agent_starting_period": v["max_agent_starting_period"],
        "preemptible": bool(v["preemptible"]), "name_prefix": _name(cid, "agent-"),
        "labels": {LABEL: cid},
        "network_interface": {"network": f"projects/{v['project_id']}/global/networks/{_name(cid, 'net')}",
                              "subnetwork": f"projects/{v['project_id']}/regions/{v['region']}/subnetworks/{_name(cid, 'subnet')}",
                              "external_ip": True},
        "service_account": {"email": "SERVICE_ACCOUNT_EMAIL"},
    }
    return {"host": "0.0.0.0", "port": v["port"], "external_url": "http://MASTER_IP:%d" % v["port"],
            "cluster_name": cid,
            "checkpoint_storage": {"type": "gcs", "bucket": v["bucket"]},
            "resource_manager": {"type": "agent", "scheduler": {"type": v["scheduler_type"],
                                                                "preemption": bool(v["preemption_enabled"])}},
            "resource_pools": [{"pool_name": "default", "provider": provider}]}


def startup_script(v: Dict[str, Any]) -> str:
    # Terraform interpolates ${...}: literal shell variables are written $${...}
    cfg = yaml.safe_dump(master_yaml(v), sort_keys=False)
    cfg = cfg.replace("SERVICE_ACCOUNT_EMAIL", "${google_service_account.det.email}").replace("MASTER_IP", "$${IP}")
    return "\n".join([
        "#!/bin/bash", "set -ex", "mkdir -p /etc/determined /var/lib/determined",
        'IP=$(curl -s -H "Metadata-Flavor: Google" '
        "http://metadata.google.internal/computeMetadata/v1/instance/network-interfaces/0/ip)",
        "cat > /etc/determined/master.yaml <<EOF", cfg.rstrip(), "EOF",
        "cat > /etc/systemd/system/determined-master.service <<EOF",
        "[Unit]", "Description=determined_clone_amd master", "After=network-online.target", "[Service]",
        "Environment=HSA_ENABLE_IPC_MODE_LEGACY=0",
        "ExecStart=/usr/bin/python3 -m determined_clone_amd.master --config-file /etc/determined/master.yaml "
        "--db /var/lib/determined/master.db",
        "Restart=always", "[Install]", "WantedBy=multi-user.target", "EOF",
        "systemctl daemon-reload", "systemctl enable --now determined-master", ""])


def terraform_config(v: Dict[str, Any]) -> Dict[str, Any]:
    cid, project, region, zone = v["cluster_id"], v["project_id"], v["region"], v["zone"]
    sa = "serviceAccount:${google_service_account.det.email}"
    tag = _name(cid, "master")
    cfg: Dict[str, Any] = {
        "terraform": {"required_providers": {"google": {"source": "hashicorp/google"}}},
        "provider": {"google": {"project": project, "region": region, "zone": zone}},
        "resource": {
            "google_compute_network": {"det": {"name": _name(cid, "net"), "auto_create_subnetworks": False}},
            "google_compute_subnetwork": {"det": {"name": _name(cid, "subnet"), "region": region,
                                                  "ip_cidr_range": v["subnet_cidr"],
                                                  "network": "${google_compute_network.det.id}"}},
            "google_compute_firewall": {
                "master": {"name": _name(cid, "master-fw"), "network": "${google_compute_network.det.name}",
                           "allow": [{"protocol": "tcp", "ports": [str(v["port"]), "22"]}],
                           "source_ranges": [v["inbound_cidr"]], "target_tags": [tag]},
                # master <-> agents and agent <-> agent (RCCL) on every port inside the subnet
                "internal": {"name": _name(cid, "internal-fw"), "network": "${google_compute_network.det.name}",
                             "allow": [{"protocol": "tcp"}, {"protocol": "udp"}, {"protocol": "icmp"}],
                             "source_ranges": [v["subnet_cidr"]]},
            },
            "google_service_account": {"det": {"account_id": _name(cid, "sa")[:30].rstrip("-"),
                                               "display_name": f"determined cluster {cid}"}},
            "google_project_iam_member": {
                role.split("/")[1].replace(".", "_"): {"project": project, "role": role, "member": sa}
                for role in ("roles/compute.instanceAdmin.v1", "roles/iam.serviceAccountUser",
                             "roles/storage.objectAdmin", "roles/logging.logWriter")},
            "google_storage_bucket": {"checkpoints": {"name": v["bucket"], "location": region,
                                                      "uniform_bucket_level_access": True,
                                                      "force_destroy": False, "labels": {LABEL: cid}}},
            "google_compute_address": {"master": {"name": _name(cid, "master-ip"), "region": region}},
            "google_compute_instance": {"master": {
                "name": tag, "machine_type": v["master_instance_type"], "zone": zone, "tags": [tag],
                "labels": {LABEL: cid},
                "boot_disk": {"initialize_params": {"image": v["environment_image"], "size": 200}},
                "network_interface": [{"subnetwork": "${google_compute_subnetwork.det.id}",
                                       "access_config": [{"nat_ip": "${google_compute_address.master.address}"}]}],
                "service_account": {"email": "${google_service_account.det.email}", "scopes": ["cloud-platform"]},
                "metadata_startup_script": startup_script(v),
                "depends_on": ["google_project_iam_member.compute_instanceAdmin_v1"],
            }},
        },
        "output": {
            "master_url": {"value": "http://${google_compute_address.master.address}:%d" % v["port"]},
            "checkpoint_bucket": {"value": "${google_storage_bucket.checkpoints.name}"},
            "service_account": {"value": "${google_service_account.det.email}"},
        },
    }
    if v.get("tf_state_gcs_bucket_name"):
        cfg["terraform"]["backend"] = {"gcs": {"bucket": v["tf_state_gcs_bucket_name"], "prefix": f"determined/{cid}"}}
    return cfg


DEFAULTS: Dict[str, Any] = {
    "region": "us-central1", "zone": None, "port": 8080, "inbound_cidr": "0.0.0.0/0",
    "subnet_cidr": "10.20.0.0/16", "master_instance_type": "n2-standard-4",
    "gpu_agent_instance_type": None, "gpu_type": None, "gpu_num": 8, "disk_size": 500,
    "environment_image": None, "preemptible": False, "min_dynamic_agents": 0, "max_dynamic_agents": 4,
    "max_idle_agent_period": "10m", "max_agent_starting_period": "20m", "scheduler_type": "priority",
    "preemption_enabled": True, "bucket": None, "tf_state_gcs_bucket_name": None,
}


def values(args: Any) -> Dict[str, Any]:
    v = dict(DEFAULTS)
    for k in list(DEFAULTS) + ["cluster_id", "project_id"]:
        x = getattr(args, k, None)
        if x is not None:
            v[k] = x
    v["zone"] = v["zone"] or f"{v['region']}-a"
    v["bucket"] = v["bucket"] or f"{v['project_id']}-det-{v['cluster_id']}-checkpoints"
    for req in ("cluster_id", "project_id", "environment_image", "gpu_agent_instance_type"):
        if not v.get(req):
            raise ValueError(f"--{req.replace('_', '-')} is required")
    return v


def state_dir(args: Any) -> str:
    base = getattr(args, "local_state_path", None) or os.path.join(os.path.expanduser("~"), ".det-clone", "gcp")
    return os.path.join(base, args.cluster_id)


def terraform(args_list: List[str], cwd: str, bin_: str = "terraform") -> None:
    try:
        subprocess.run([bin_] + args_list, cwd=cwd, check=True)
    except FileNotFoundError:
        raise RuntimeError(f"{bin_} not found on PATH: install Terraform or use --dry-run")
    except subprocess.CalledProcessError as e:
        raise RuntimeError(f"terraform {' '.join(args_list)} failed with exit code {e.returncode}")


def write_config(args: Any) -> str:
    d = state_dir(args)
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, "main.tf.json"), "w") as f:
        json.dump(terraform_config(values(args)), f, indent=2)
    return d


def up(args: Any, log: Callable[[str], None] = print, tf_bin: str = "terraform") -> Optional[Dict[str, Any]]:
    d = write_config(args)
    log(f"terraform configuration: {os.path.join(d, 'main.tf.json')}")
    if getattr(args, "dry_run", False):
        return None
    terraform(["init", "-input=false"], d, tf_bin)
    terraform(["apply", "-input=false", "-auto-approve"], d, tf_bin)
    out = subprocess.run([tf_bin, "output", "-json"], cwd=d, capture_output=True, text=True, check=True).stdout
    res = {k: x.get("value") for k, x in json.loads(out or "{}").items()}
    if res.get("master_url"):
        log(f"master: {res['master_url']}")
    return res


def down(args: Any, log: Callable[[str], None] = print, tf_bin: str = "terraform", gce: Any = None) -> None:
    d = state_dir(args)
    if not os.path.exists(os.path.join(d, "main.tf.json")):
        raise RuntimeError(f"no deployment state in {d}")
    v = json.load(open(os.path.join(d, "main.tf.json")))
    # agents were created by the master's provisioner (not by Terraform): delete them first
    if gce is None:
        from determined_clone_amd.master.provisioner import GCPProvider

        prov = v["provider"]["google"]
        gce = GCPProvider("default", {"project": prov["project"], "zone": prov["zone"],
                                      "endpoint_url": getattr(args, "compute_endpoint_url", None)}, "http://unused:0")
        gce.labels = {LABEL: args.cluster_id}
    agents = [i.id for i in gce.list()
              if not i.id.endswith("-master")]
    if agents:
        gce.terminate(agents)
        log(f"deleted {len(agents)} agent instance(s)")
    # like `det deploy aws down`, keep the checkpoints: forget the bucket, then destroy the rest
    subprocess.run([tf_bin, "state", "rm", "google_storage_bucket.checkpoints"], cwd=d,
                   capture_output=True, check=False)
    terraform(["destroy", "-input=false", "-auto-approve"], d, tf_bin)
    log(f"cluster {args.cluster_id} destroyed (checkpoint bucket {v['resource']['google_storage_bucket']['checkpoints']['name']} kept)")


def list_clusters(args: Any) -> List[str]:
    base = getattr(args, "local_state_path", None) or os.path.join(os.path.expanduser("~"), ".det-clone", "gcp")
    return sorted(x for x in os.listdir(base) if os.path.exists(os.path.join(base, x, "main.tf.json"))) \
        if os.path.isdir(base) else []
