"""Dynamic agents: a resource pool's provisioner launches and terminates cloud instances (MI355X
VMs) that run this framework's agent.

Reference: `master/internal/rm/agentrm/provisioner/` (`provisioner.go`, `scaledecider/`,
`aws/aws.go`, `gcp/gcp.go`, `agentsetup/`) and `agentrm/scaling.go`. The pieces:

* :func:`desired_new_instances` -- how many instances the pool's unscheduled requests need
  (`scaling.go: calculateDesiredNewAgentNum`): slots summed over requests a single instance can
  host (``slots <= slots_per_instance`` or a multiple of it), zero-slot tasks packed
  ``max_zero_slot_tasks_per_agent`` per instance, the larger of the two instance counts;
* :class:`ScaleDecider` -- instance bookkeeping (`scale_decider.go`): pending / recently launched /
  idle / disconnected / stopped instances and their timers; terminates stopped ones, ones
  disconnected past ``max_disconnect_period``, ones idle past ``max_idle_agent_period`` (down to
  ``min_instances``) and anything above ``max_instances`` (pending spot requests first, then idle,
  disconnected, newest); launches ``clamp(min - n, desired - recently_launched, max - n)``;
* :class:`Provisioner` -- one provisioning tick every ``action_cooldown`` s (list -> decide ->
  terminate -> launch), launch errors sticky for ``launch_error_timeout``;
* providers -- :class:`AWSProvider` (EC2 Query API signed with SigV4: DescribeInstances filtered by
  the cluster tag + pool tag, RunInstances with the agent-setup user data, TerminateInstances) and
  :class:`GCPProvider` (Compute Engine REST: instances.list filtered by labels, bulkInsert,
  delete), both over plain HTTPS (no cloud SDKs in the image);
* :func:`agent_setup_script` -- the instance's startup script: starts this framework's agent with
  the master address, the pool and the instance id as the agent id (so the decider can associate
  connected agents with instances).
"""
import base64
import datetime
import hashlib
import logging
import re
import threading
import time
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Any, Callable, Dict, List, Optional

import requests

from determined_clone_amd.common.storage._cloud import imds_credentials, sigv4_headers

logger = logging.getLogger("determined_clone_amd.master.provisioner")

# instance states (reference: master/pkg/model/instance.go)
STARTING, RUNNING, STOPPING, STOPPED, TERMINATING, UNKNOWN, SPOT_PENDING = (
    "Starting", "Running", "Stopping", "Stopped", "Terminating", "Unknown", "SpotRequestPendingAWS")

TERMINATE_STOPPED = "instance is stopped"
TERMINATE_LONG_DISCONNECTED = "instance has been disconnected for a long time"
TERMINATE_LONG_IDLE = "instance has been idle for a long time"
TERMINATE_EXCEEDS_MAX = "instance number exceeds the maximum"


class Instance:
    __slots__ = ("id", "agent_name", "state", "launch_time", "last_state_change")

    def __init__(self, id: str, agent_name: str, state: str, launch_time: float) -> None:
        self.id, self.agent_name, self.state, self.launch_time = id, agent_name, state, launch_time
        self.last_state_change = time.time()

    def key(self) -> tuple:
        return (self.id, self.agent_name, self.state, self.launch_time)

    def __repr__(self) -> str:
        return f"Instance({self.id}, {self.state})"


def desired_new_instances(pending: List[Any], slots_per_instance: int,
                          max_zero_slot_tasks_per_agent: int = 100,
                          max_slots: Optional[Dict[str, int]] = None) -> int:
    """Instances needed by the unscheduled requests ``pending`` (objects with ``slots`` and
    ``job_id``); ``max_slots`` caps the slots counted per job (expconf resources.max_slots)."""
    zero = 0
    per_job: Dict[str, int] = {}
    for r in pending:
        if r.slots == 0:
            zero += 1
        elif slots_per_instance == 0:
            continue
        elif r.slots <= slots_per_instance or r.slots % slots_per_instance == 0:
            per_job[r.job_id] = per_job.get(r.job_id, 0) + r.slots
    slot_sum = 0
    for job, s in per_job.items():
        cap = (max_slots or {}).get(job)
        slot_sum += min(cap, s) if cap is not None else s
    by_zero = -(-zero // max_zero_slot_tasks_per_agent) if zero and max_zero_slot_tasks_per_agent else 0
    by_slot = -(-slot_sum // slots_per_instance) if slot_sum and slots_per_instance else 0
    return max(by_zero, by_slot)


class ScaleDecider:
    def __init__(self, max_idle_period: float, max_starting_period: float,
                 max_disconnect_period: float, min_instances: int, max_instances: int,
                 clock: Callable[[], float] = time.time) -> None:
        self.max_idle = max_idle_period
        self.max_starting = max_starting_period
        self.max_disconnect = max_disconnect_period
        self.min_instances = min_instances
        self.max_instances = max_instances
        self.clock = clock
        self.snapshot: Optional[Dict[str, Instance]] = None
        self.connected: Dict[str, Any] = {}
        self.idle_agents: Dict[str, Any] = {}
        self.desired = 0
        self.instances: Dict[str, Instance] = {}
        self.pending: Dict[str, bool] = {}
        self.recently_launched: Dict[str, bool] = {}
        self.stopped: Dict[str, bool] = {}
        self.disconnected: Dict[str, float] = {}
        self.idle: Dict[str, float] = {}
        self.long_disconnected: Dict[str, bool] = {}
        self.long_idle: Dict[str, bool] = {}
        self._lock = threading.Lock()

    def update_scaling_info(self, desired_new: int, agents: List[Dict[str, Any]]) -> None:
        """``agents``: connected agents of the pool as ``{"name": str, "idle": bool}``."""
        with self._lock:
            self.desired = desired_new
            self.connected = {a["name"]: a for a in agents}
            self.idle_agents = {a["name"]: a for a in agents if a.get("idle")}

    def update_instance_snapshot(self, instances: List[Instance]) -> bool:
        with self._lock:
            old = self.snapshot
            changed = old is None or len(old) != len(instances) or any(
                i.id not in old or old[i.id].key() != i.key() for i in instances)
            if changed:
                now = self.clock()
                for inst in instances:
                    prev = (old or {}).get(inst.id)
                    inst.last_state_change = now if prev is None or prev.state != inst.state else prev.last_state_change
                self.snapshot = {i.id: i for i in instances}
            return changed

    def calculate_instance_states(self) -> None:
        with self._lock:
            now = self.clock()
            past_disc, past_idle = self.disconnected, self.idle
            self.instances, self.pending, self.recently_launched, self.stopped = {}, {}, {}, {}
            self.disconnected, self.idle, self.long_disconnected, self.long_idle = {}, {}, {}, {}
            for inst in (self.snapshot or {}).values():
                if inst.state == SPOT_PENDING:
                    self.instances[inst.id] = inst
                    self.pending[inst.id] = True
                    self.recently_launched[inst.id] = True
                elif inst.state in (STARTING, RUNNING):
                    self.instances[inst.id] = inst
                    if inst.agent_name in self.connected:
                        if inst.agent_name in self.idle_agents:
                            t = past_idle.get(inst.id)
                            if t is not None:
                                if now > t + self.max_idle:
                                    self.long_idle[inst.id] = True
                                self.idle[inst.id] = t
                            else:
                                self.idle[inst.id] = now
                        continue
                    if inst.launch_time + self.max_starting > now:
                        self.recently_launched[inst.id] = True
                        continue
                    t = past_disc.get(inst.id)
                    if t is not None:
                        if now > t + self.max_disconnect:
                            self.long_disconnected[inst.id] = True
                        self.disconnected[inst.id] = t
                    else:
                        self.disconnected[inst.id] = now
                elif inst.state == STOPPED:
                    self.stopped[inst.id] = True

    def find_instances_to_terminate(self) -> Dict[str, str]:
        with self._lock:
            out: Dict[str, str] = {}
            for i in list(self.stopped):
                out[i] = TERMINATE_STOPPED
                del self.stopped[i]
            for i in list(self.long_disconnected):
                out[i] = TERMINATE_LONG_DISCONNECTED
                self.disconnected.pop(i, None)
            for i in sorted(self.long_idle):
                if len(self.instances) - len(out) > self.min_instances:
                    out[i] = TERMINATE_LONG_IDLE
                    self.idle.pop(i, None)
                else:
                    break
            for group in (self.pending, self.idle, self.disconnected):
                for i in sorted(group):
                    if len(self.instances) - len(out) > self.max_instances:
                        out[i] = TERMINATE_EXCEEDS_MAX
                        group.pop(i, None)
                    else:
                        break
            newest_first = sorted(self.instances.values(), key=lambda x: -x.launch_time)
            for inst in newest_first:
                if len(self.instances) - len(out) <= self.max_instances:
                    break
                out.setdefault(inst.id, TERMINATE_EXCEEDS_MAX)
            return out

    def num_instances_to_launch(self) -> int:
        with self._lock:
            n = len(self.instances)
            # mathx.Clamp(lo, v, hi) = min(max(lo, v), hi)
            v = min(max(self.min_instances - n, self.desired - len(self.recently_launched)),
                    self.max_instances - n)
            return max(0, v)


def agent_setup_script(master_url: str, resource_pool: str, agent_id_cmd: str,
                       startup_script: str = "", agent_args: str = "",
                       python: str = "python3") -> str:
    """Startup script of a provisioned instance: run the user's startup script, then this
    framework's agent (reference: `agentsetup` + `master/static/srv/agent_setup_script.sh.template`)."""
    return "\n".join([
        "#!/bin/bash",
        "set -x",
        "export HSA_ENABLE_IPC_MODE_LEGACY=0",
        startup_script or ":",
        f'AGENT_ID="{agent_id_cmd}"',
        f"exec {python} -m determined_clone_amd.agent --master-url {master_url} "
        f"--resource-pool {resource_pool} --agent-id \"$AGENT_ID\" {agent_args}".rstrip(),
        "",
    ])


class Provider:
    slots_per_instance = 0
    instance_type = ""

    def list(self) -> List[Instance]:
        raise NotImplementedError

    def launch(self, n: int) -> None:
        raise NotImplementedError

    def terminate(self, ids: List[str]) -> None:
        raise NotImplementedError


# ----------------------------------------------------------------------------------------- AWS
EC2_STATES = {"pending": STARTING, "running": RUNNING, "stopped": STOPPED, "stopping": STOPPING,
              "shutting-down": TERMINATING}


def _xml_items(el: Optional[ET.Element], tag: str) -> List[ET.Element]:
    return [] if el is None else [c for c in el if _local(c.tag) == tag]


def _local(tag: str) -> str:
    return tag.split("}", 1)[-1]


def _find(el: ET.Element, *path: str) -> Optional[ET.Element]:
    cur: Optional[ET.Element] = el
    for p in path:
        if cur is None:
            return None
        cur = next((c for c in cur if _local(c.tag) == p), None)
    return cur


def _text(el: ET.Element, *path: str) -> str:
    e = _find(el, *path)
    return (e.text or "") if e is not None else ""


def _iso(ts: str) -> float:
    try:
        return datetime.datetime.fromisoformat(ts.replace("Z", "+00:00")).timestamp()
    except ValueError:
        return time.time()


class AWSProvider(Provider):
    """On-demand EC2 instances tagged ``<tag_key>=<tag_value>`` + ``determined-resource-pool``."""

    def __init__(self, pool: str, config: Dict[str, Any], master_url: str,
                 session: Optional[requests.Session] = None) -> None:
        import os

        self.pool = pool
        self.cfg = config
        self.region = config.get("region", "us-east-1")
        self.endpoint = config.get("endpoint_url") or f"https://ec2.{self.region}.amazonaws.com/"
        self.access_key = config.get("access_key") or os.environ.get("AWS_ACCESS_KEY_ID", "")
        self.secret_key = config.get("secret_key") or os.environ.get("AWS_SECRET_ACCESS_KEY", "")
        self.token = os.environ.get("AWS_SESSION_TOKEN")
        self.imds = (config.get("imds_endpoint") or "http://169.254.169.254").rstrip("/")
        self._imds_expiry = 0.0
        self.tag_key = config.get("tag_key", "determined-clone-amd")
        self.tag_value = config.get("tag_value", "determined-clone-amd-agent")
        self.instance_type = (config.get("instance_type") or {}).get("name", "") \
            if isinstance(config.get("instance_type"), dict) else config.get("instance_type", "")
        self.slots_per_instance = int(config.get("slots_per_instance", 8))
        self.master_url = master_url
        self.http = session or requests.Session()
        self.user_data = agent_setup_script(
            master_url, pool, "$(curl -s http://169.254.169.254/latest/meta-data/instance-id)",
            config.get("startup_script", ""), config.get("agent_args", ""))

    def _refresh_credentials(self) -> None:
        """No static keys: use the instance profile of the machine the master runs on (IMDSv2),
        which is how ``det deploy aws`` grants the master its EC2 permissions."""
        if (self.access_key and not self._imds_expiry) or \
                (self._imds_expiry and time.time() < self._imds_expiry - 300):
            return
        c = imds_credentials(self.http, self.imds)
        self.access_key, self.secret_key, self.token = c["access_key"], c["secret_key"], c["token"]
        self._imds_expiry = c["expiry"]

    def _call(self, action: str, params: Dict[str, str]) -> ET.Element:
        self._refresh_credentials()
        body = urllib.parse.urlencode({"Action": action, "Version": "2016-11-15", **params})
        sha = hashlib.sha256(body.encode()).hexdigest()
        h = sigv4_headers("POST", self.endpoint,
                          {"content-type": "application/x-www-form-urlencoded; charset=utf-8"},
                          sha, self.access_key, self.secret_key, self.region, "ec2",
                          session_token=self.token)
        r = self.http.post(self.endpoint, data=body, headers=h, timeout=60)
        if r.status_code >= 300:
            raise RuntimeError(f"EC2 {action}: HTTP {r.status_code}: {r.text[:300]}")
        return ET.fromstring(r.content)

    def _instances(self, root: ET.Element) -> List[Instance]:
        out = []
        for rsv in _xml_items(_find(root, "reservationSet"), "item"):
            for it in _xml_items(_find(rsv, "instancesSet"), "item"):
                iid = _text(it, "instanceId")
                st = EC2_STATES.get(_text(it, "instanceState", "name"), UNKNOWN)
                out.append(Instance(iid, iid, st, _iso(_text(it, "launchTime"))))
        return out

    def list(self) -> List[Instance]:
        params = {"Filter.1.Name": f"tag:{self.tag_key}", "Filter.1.Value.1": self.tag_value,
                  "Filter.2.Name": "tag:determined-resource-pool", "Filter.2.Value.1": self.pool,
                  "Filter.3.Name": "instance-state-name", "Filter.3.Value.1": "running",
                  "Filter.3.Value.2": "pending", "Filter.3.Value.3": "stopped"}
        return self._instances(self._call("DescribeInstances", params))

    def launch(self, n: int) -> None:
        c = self.cfg
        tags = [("Name", c.get("instance_name", "determined-clone-amd-agent")),
                (self.tag_key, self.tag_value), ("determined-resource-pool", self.pool),
                ("determined-master-address", self.master_url)]
        tags += [(t["key"], t["value"]) for t in c.get("custom_tags") or []]
        params = {
            "ImageId": c.get("image_id", ""), "InstanceType": self.instance_type,
            "MinCount": "1", "MaxCount": str(n), "InstanceInitiatedShutdownBehavior": "terminate",
            "UserData": base64.b64encode(self.user_data.encode()).decode(),
            "BlockDeviceMapping.1.DeviceName": "/dev/sda1",
            "BlockDeviceMapping.1.Ebs.DeleteOnTermination": "true",
            "BlockDeviceMapping.1.Ebs.VolumeSize": str(c.get("root_volume_size", 200)),
            "BlockDeviceMapping.1.Ebs.VolumeType": "gp2",
            "MetadataOptions.HttpTokens": "required", "MetadataOptions.HttpPutResponseHopLimit": "2",
            "TagSpecification.1.ResourceType": "instance",
        }
        for i, (k, v) in enumerate(tags, 1):
            params[f"TagSpecification.1.Tag.{i}.Key"] = k
            params[f"TagSpecification.1.Tag.{i}.Value"] = v
        if c.get("ssh_key_name"):
            params["KeyName"] = c["ssh_key_name"]
        if c.get("iam_instance_profile_arn"):
            params["IamInstanceProfile.Arn"] = c["iam_instance_profile_arn"]
        if (c.get("network_interface") or {}).get("subnet_id"):
            params["SubnetId"] = c["network_interface"]["subnet_id"]
        if (c.get("network_interface") or {}).get("security_group_id"):
            params["SecurityGroupId.1"] = c["network_interface"]["security_group_id"]
        self._call("RunInstances", params)

    def terminate(self, ids: List[str]) -> None:
        if ids:
            self._call("TerminateInstances", {f"InstanceId.{i}": x for i, x in enumerate(ids, 1)})


# ----------------------------------------------------------------------------------------- GCP
GCE_STATES = {"PROVISIONING": STARTING, "STAGING": STARTING, "RUNNING": RUNNING,
              "STOPPING": STOPPING, "SUSPENDING": STOPPING, "STOPPED": STOPPED,
              "SUSPENDED": STOPPED, "TERMINATED": STOPPED}


class GCPProvider(Provider):
    """Compute Engine instances labelled with the master host/port and the pool."""

    def __init__(self, pool: str, config: Dict[str, Any], master_url: str,
                 session: Optional[requests.Session] = None) -> None:
        import os

        self.pool = pool
        self.cfg = config
        self.project, self.zone = config["project"], config["zone"]
        self.endpoint = (config.get("endpoint_url") or "https://compute.googleapis.com/compute/v1").rstrip("/")
        self.token = config.get("token") or os.environ.get("GCE_ACCESS_TOKEN", "")
        self.metadata = (config.get("metadata_endpoint") or "http://metadata.google.internal").rstrip("/")
        self._token_expiry = 0.0
        self.instance_type = (config.get("instance_type") or {}).get("machine_type", "")
        self.slots_per_instance = int(config.get("slots_per_instance",
                                                 (config.get("instance_type") or {}).get("gpu_num", 8)))
        self.name_prefix = config.get("name_prefix", "det-agent-")
        u = urllib.parse.urlsplit(master_url)
        self.labels = {"determined-master-host": (u.hostname or "").replace(".", "-"),
                       "determined-master-port": str(u.port or ""),
                       "determined-resource-pool": pool}
        self.http = session or requests.Session()
        self.startup = agent_setup_script(
            master_url, pool,
            '$(curl -s "http://metadata.google.internal/computeMetadata/v1/instance/name" '
            '-H "Metadata-Flavor: Google")', config.get("startup_script", ""), config.get("agent_args", ""))

    def _refresh_token(self) -> None:
        """No configured token: the service account of the VM the master runs on (metadata
        server), which is how ``det deploy gcp`` grants the master its Compute permissions."""
        if self.token and not self._token_expiry:
            return
        if self._token_expiry and time.time() < self._token_expiry - 300:
            return
        d = self.http.get(f"{self.metadata}/computeMetadata/v1/instance/service-accounts/default/token",
                          headers={"Metadata-Flavor": "Google"}, timeout=5).json()
        self.token = d["access_token"]
        self._token_expiry = time.time() + float(d.get("expires_in", 3600))

    def _req(self, method: str, path: str, **kw: Any) -> Any:
        self._refresh_token()
        r = self.http.request(method, f"{self.endpoint}/projects/{self.project}/zones/{self.zone}{path}",
                              headers={"Authorization": f"Bearer {self.token}"}, timeout=60, **kw)
        if r.status_code >= 300:
            raise RuntimeError(f"GCE {method} {path}: HTTP {r.status_code}: {r.text[:300]}")
        return r.json() if r.content else {}

    def list(self) -> List[Instance]:
        flt = " AND ".join(f"(labels.{k} = {v})" for k, v in self.labels.items())
        out = []
        token = None
        while True:
            params = {"filter": flt}
            if token:
                params["pageToken"] = token
            d = self._req("GET", "/instances", params=params)
            for it in d.get("items") or []:
                out.append(Instance(it["name"], it["name"], GCE_STATES.get(it.get("status", ""), UNKNOWN),
                                    _iso(it.get("creationTimestamp", ""))))
            token = d.get("nextPageToken")
            if not token:
                return out

    def launch(self, n: int) -> None:
        c = self.cfg
        props = {
            "machineType": self.instance_type,
            "labels": dict(self.labels, **(c.get("labels") or {})),
            "metadata": {"items": [{"key": "startup-script", "value": self.startup}]},
            "disks": [{"boot": True, "autoDelete": True, "initializeParams": {
                "sourceImage": c.get("boot_disk_source_image", ""),
                "diskSizeGb": str(c.get("boot_disk_size", 200))}}],
            "networkInterfaces": [{"network": c.get("network_interface", {}).get("network", "global/networks/default"),
                                   "subnetwork": c.get("network_interface", {}).get("subnetwork", "")}],
            "scheduling": {"onHostMaintenance": "TERMINATE", "preemptible": bool(c.get("preemptible", False))},
        }
        if c.get("service_account"):  # the agents' identity (checkpoint bucket access)
            sa = c["service_account"]
            props["serviceAccounts"] = [{"email": sa.get("email", "default"),
                                         "scopes": sa.get("scopes") or ["https://www.googleapis.com/auth/cloud-platform"]}]
        if c.get("network_interface", {}).get("external_ip", True):
            props["networkInterfaces"][0]["accessConfigs"] = [{"type": "ONE_TO_ONE_NAT", "name": "External NAT"}]
        if c.get("instance_type", {}).get("gpu_type"):
            props["guestAccelerators"] = [{"acceleratorType": c["instance_type"]["gpu_type"],
                                           "acceleratorCount": self.slots_per_instance}]
        body = {"count": str(n), "namePattern": self.name_prefix + "#" * 8, "instanceProperties": props}
        self._req("POST", "/instances/bulkInsert", json=body)

    def terminate(self, ids: List[str]) -> None:
        for name in ids:
            try:
                self._req("DELETE", f"/instances/{name}")
            except Exception as e:
                logger.warning(f"could not delete instance {name}: {e}")


# ----------------------------------------------------------------------------------------- loop
class Provisioner:
    def __init__(self, pool: str, config: Dict[str, Any], provider: Provider,
                 clock: Callable[[], float] = time.time,
                 scaling_info: Optional[Callable[[], Any]] = None) -> None:
        self.pool = pool
        self.provider = provider
        # () -> (unscheduled requests of the pool, [{"name": agent id, "idle": bool}])
        self.scaling_info = scaling_info
        self.decider = ScaleDecider(
            _seconds(config.get("max_idle_agent_period", "20m")),
            _seconds(config.get("max_agent_starting_period", "20m")),
            _seconds(config.get("max_disconnect_period", "10m")),
            int(config.get("min_instances", 0)), int(config.get("max_instances", 5)), clock)
        self.max_zero_slot = int(config.get("max_zero_slot_tasks_per_agent", 100))
        self.cooldown = _seconds(config.get("action_cooldown", "5s"))
        self.launch_error_timeout = _seconds(config.get("launch_error_timeout", "0s"))
        self.launch_error: Optional[str] = None
        self.launch_error_at = 0.0
        self.clock = clock
        self.history: List[Dict[str, Any]] = []
        self._stop = threading.Event()
        self._lock = threading.Lock()

    def update_scaling_info(self, pending: List[Any], agents: List[Dict[str, Any]]) -> None:
        self.decider.update_scaling_info(
            desired_new_instances(pending, self.provider.slots_per_instance, self.max_zero_slot), agents)

    def provision(self) -> None:
        with self._lock:
            if self.scaling_info is not None:
                self.update_scaling_info(*self.scaling_info())
            try:
                instances = self.provider.list()
            except Exception as e:
                logger.error(f"pool {self.pool}: cannot list instances: {e}")
                return
            if self.decider.update_instance_snapshot(instances):
                logger.info(f"pool {self.pool}: instances {instances}")
            self.decider.calculate_instance_states()
            term = self.decider.find_instances_to_terminate()
            if term:
                logger.info(f"pool {self.pool}: terminating {term}")
                self.history.append({"terminate": dict(term), "time": self.clock()})
                try:
                    self.provider.terminate(sorted(term))
                except Exception as e:
                    logger.error(f"pool {self.pool}: terminate failed: {e}")
            n = self.decider.num_instances_to_launch()
            if n > 0:
                if self.launch_error and self.clock() < self.launch_error_at + self.launch_error_timeout:
                    return
                logger.info(f"pool {self.pool}: launching {n} instance(s) of {self.provider.instance_type}")
                self.history.append({"launch": n, "time": self.clock()})
                try:
                    self.provider.launch(n)
                    self.launch_error = None
                except Exception as e:
                    self.launch_error, self.launch_error_at = str(e), self.clock()
                    logger.error(f"pool {self.pool}: launch failed: {e}")

    def run(self) -> None:
        while not self._stop.wait(self.cooldown):
            self.provision()

    def start(self) -> "Provisioner":
        threading.Thread(target=self.run, daemon=True, name=f"provisioner-{self.pool}").start()
        return self

    def stop(self) -> None:
        self._stop.set()


def _seconds(v: Any) -> float:
    """Go-style duration ("20m", "5s", "1h30m", "300ms") or a number of seconds."""
    if isinstance(v, (int, float)):
        return float(v)
    total = 0.0
    for num, unit in re.findall(r"([0-9.]+)(ms|s|m|h)", str(v)):
        total += float(num) * {"ms": 1e-3, "s": 1.0, "m": 60.0, "h": 3600.0}[unit]
    return total


def make_provider(pool: str, provider_cfg: Dict[str, Any], master_url: str) -> Provider:
    t = provider_cfg.get("type")
    if t == "aws":
        return AWSProvider(pool, provider_cfg, master_url)
    if t == "gcp":
        return GCPProvider(pool, provider_cfg, master_url)
    raise ValueError(f"unknown provider type {t!r} (aws | gcp)")
