"""Cloud / Kubernetes deployment (reference: `harness/determined/deploy/{aws,gcp,gke}`,
`helm/charts/determined`). No cloud here: the CloudFormation query API, EC2, GCE, the EC2
metadata service, ``kubectl``, ``terraform`` and ``gcloud`` are fakes; what is checked is what
would be sent to them and that the generated configurations are internally consistent."""
import argparse
import json
import os
import re
import stat
import threading
import urllib.parse
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest
import yaml

from determined_clone_amd.cli.cli import build_parser
from determined_clone_amd.deploy import aws, gcp, gke
from determined_clone_amd.deploy import kubernetes as k8s
from determined_clone_amd.deploy.healthcheck import wait_for_master

from fake_cluster import FakeEC2, FakeGCE


class _Srv:
    def __init__(self, handle):
        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def _go(self, method):
                n = int(self.headers.get("Content-Length") or 0)
                code, body, ctype = handle(method, self.path, self.rfile.read(n) if n else b"", self.headers)
                data = body if isinstance(body, bytes) else body.encode()
                self.send_response(code)
                self.send_header("Content-Type", ctype)
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

            do_GET = lambda self: self._go("GET")  # noqa: E731
            do_PUT = lambda self: self._go("PUT")  # noqa: E731
            do_POST = lambda self: self._go("POST")  # noqa: E731

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.httpd.server_address[1]}"
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


def _script(path, body):
    with open(path, "w") as f:
        f.write("#!/bin/bash\n" + body)
    os.chmod(path, os.stat(path).st_mode | stat.S_IEXEC)
    return str(path)


# ============================================================================ Kubernetes
def test_k8s_render_consistent():
    ms = k8s.render({"namespace": "det-ns", "image": "reg/det:1", "storage_class": "fast"})
    kinds = [m["kind"] for m in ms]
    for k in ("Namespace", "ServiceAccount", "Role", "RoleBinding", "ClusterRole", "ClusterRoleBinding",
              "ConfigMap", "PersistentVolumeClaim", "Deployment", "Service"):
        assert k in kinds, k
    assert all(m["metadata"].get("namespace", "det-ns") == "det-ns" for m in ms if m["kind"] not in ("ClusterRole", "ClusterRoleBinding"))
    cfg = yaml.safe_load(next(m for m in ms if m["kind"] == "ConfigMap")["data"]["master.yaml"])
    rm = cfg["resource_manager"]
    assert rm["type"] == "kubernetes" and rm["namespace"] == "det-ns" and rm["slot_resource"] == "amd.com/gpu"
    assert rm["max_slots_per_pod"] == 8 and rm["default_image"] == "reg/det:1"
    assert cfg["external_url"] == "http://det-master.det-ns.svc.cluster.local:8080"
    assert cfg["checkpoint_storage"] == {"type": "shared_fs", "host_path": "/determined/checkpoints"}
    dep = next(m for m in ms if m["kind"] == "Deployment")
    pod = dep["spec"]["template"]["spec"]
    claims = {v["persistentVolumeClaim"]["claimName"] for v in pod["volumes"] if "persistentVolumeClaim" in v}
    pvcs = {m["metadata"]["name"] for m in ms if m["kind"] == "PersistentVolumeClaim"}
    assert claims == pvcs == {"det-db", "det-checkpoints"}
    assert all(m["spec"]["storageClassName"] == "fast" for m in ms if m["kind"] == "PersistentVolumeClaim")
    assert dep["spec"]["selector"]["matchLabels"] == dep["spec"]["template"]["metadata"]["labels"]
    svc = next(m for m in ms if m["kind"] == "Service")
    assert svc["spec"]["selector"] == dep["spec"]["selector"]["matchLabels"]
    c = pod["containers"][0]
    assert c["readinessProbe"]["httpGet"]["path"] == "/api/v1/master"
    assert pod["serviceAccountName"] == next(m for m in ms if m["kind"] == "ServiceAccount")["metadata"]["name"]
    # round-trips through YAML as a multi-document stream
    assert len(list(yaml.safe_load_all(k8s.to_yaml(ms)))) == len(ms)


def test_k8s_master_config_drives_rm_pods():
    """The rendered master.yaml builds a Kubernetes RM whose task pods mount the checkpoint PVC."""
    from determined_clone_amd.master.rm_kubernetes import KubernetesResourceManager

    cfg = k8s.master_config(k8s.merge_values({}))
    rm = KubernetesResourceManager(dict(cfg["resource_manager"], api_server="http://127.0.0.1:1"),
                                   start_watcher=False)
    pod = rm.pod_manifest({"allocation_id": "a.1", "container_rank": 0, "slots": [0, 1], "agent_id": "node-0",
                           "cluster_info": {"master_url": cfg["external_url"]}, "kind": "TRIAL"})
    c = pod["spec"]["containers"][0]
    assert c["resources"]["limits"] == {"amd.com/gpu": "2"}
    assert {"name": "checkpoints", "mountPath": "/determined/checkpoints"} in c["volumeMounts"]
    assert {"name": "checkpoints", "persistentVolumeClaim": {"claimName": "det-checkpoints"}} in pod["spec"]["volumes"]


def test_k8s_object_storage_has_no_checkpoint_pvc():
    ms = k8s.render({"checkpoint_storage": {"type": "s3", "bucket": "ckpts"}})
    assert [m["metadata"]["name"] for m in ms if m["kind"] == "PersistentVolumeClaim"] == ["det-db"]
    cfg = yaml.safe_load(next(m for m in ms if m["kind"] == "ConfigMap")["data"]["master.yaml"])
    assert cfg["checkpoint_storage"] == {"type": "s3", "bucket": "ckpts"}
    assert "task_volumes" not in cfg["resource_manager"]


def test_k8s_up_down_with_fake_kubectl(tmp_path):
    log = tmp_path / "kubectl.log"
    kb = _script(tmp_path / "kubectl", f"""echo "ARGS $*" >> {log}
if [ "$1" = apply ] || [ "$1" = delete ]; then cat >> {log}; fi
if [ "$3" = get ]; then echo '{{"status": {{"loadBalancer": {{"ingress": [{{"ip": "34.1.2.3"}}]}}}}}}'; fi
""")
    out = k8s.up({"namespace": "x"}, kubectl_bin=kb)
    assert out["master_url"] == "http://34.1.2.3:8080"
    text = log.read_text()
    assert "ARGS apply -f -" in text and "kind: Deployment" in text
    assert "ARGS -n x rollout status deployment/det-master --timeout=600s" in text
    log.write_text("")
    k8s.down({"namespace": "x"}, kubectl_bin=kb)
    text = log.read_text()
    assert "ARGS delete --ignore-not-found -f -" in text
    assert "kind: PersistentVolumeClaim" not in text.split("ARGS -n x delete pods")[0]  # volumes kept
    assert "ARGS -n x delete pods -l determined.ai/managed=true --ignore-not-found" in text


# ============================================================================ AWS
_PSEUDO = {"AWS::StackName", "AWS::Region", "AWS::AccountId", "AWS::NoValue"}


def _check_refs(tpl):
    names = set(tpl["Parameters"]) | set(tpl["Resources"]) | _PSEUDO

    def walk(x):
        if isinstance(x, dict):
            if "Ref" in x:
                assert x["Ref"] in names, x
            if "Fn::GetAtt" in x:
                assert x["Fn::GetAtt"][0] in tpl["Resources"], x
            if "Fn::Sub" in x:
                for var in re.findall(r"\$\{([^}!]+)\}", x["Fn::Sub"]):
                    assert var.split(".")[0] in names, var
            if "DependsOn" in x:
                deps = x["DependsOn"] if isinstance(x["DependsOn"], list) else [x["DependsOn"]]
                assert all(d in tpl["Resources"] for d in deps)
            for v in x.values():
                walk(v)
        elif isinstance(x, list):
            for v in x:
                walk(v)

    walk(tpl)


@pytest.mark.parametrize("kind", ["simple", "vpc"])
def test_aws_template_consistent(kind):
    tpl = aws.template(kind)
    _check_refs(tpl)
    assert ("VPC" in tpl["Resources"]) == (kind == "vpc")
    script = tpl["Resources"]["MasterInstance"]["Properties"]["UserData"]["Fn::Base64"]["Fn::Sub"]
    cfg_text = script.split("<<EOF\n", 1)[1].split("\nEOF", 1)[0]
    # every ${...} is a CloudFormation substitution; a sample substitution gives valid master YAML
    sample = re.sub(r"\$\{[^}]+\}", "x", cfg_text).replace("$IP", "10.0.0.5")
    cfg = yaml.safe_load(sample)
    prov = cfg["resource_pools"][0]["provider"]
    assert prov["type"] == "aws" and cfg["checkpoint_storage"]["type"] == "s3"
    assert ("subnet_id" in prov["network_interface"]) == (kind == "vpc")
    pol = json.dumps(tpl["Resources"]["MasterRole"])
    for action in ("ec2:RunInstances", "ec2:TerminateInstances", "ec2:DescribeInstances", "iam:PassRole"):
        assert action in pol
    with pytest.raises(ValueError):
        aws.template("lore")


class FakeCloudFormation:
    def __init__(self, key="AKIDEXAMPLE"):
        self.key = key
        self.stacks = {}
        self.calls = []
        self.srv = _Srv(self.handle)
        self.url = self.srv.url + "/"

    def handle(self, method, path, body, headers):
        auth = headers.get("Authorization") or ""
        if f"Credential={self.key}/" not in auth or "/cloudformation/aws4_request" not in auth:
            return 403, "<ErrorResponse><Error><Message>bad signature</Message></Error></ErrorResponse>", "text/xml"
        p = dict(urllib.parse.parse_qsl(body.decode()))
        self.calls.append(p)
        a, name = p["Action"], p.get("StackName")
        ns = 'xmlns="http://cloudformation.amazonaws.com/doc/2010-05-15/"'
        if a == "CreateStack":
            self.stacks[name] = {"status": ["CREATE_IN_PROGRESS", "CREATE_COMPLETE"], "params": p}
            return 200, f"<CreateStackResponse {ns}><CreateStackResult><StackId>arn:{name}</StackId></CreateStackResult></CreateStackResponse>", "text/xml"
        if a == "UpdateStack":
            self.stacks[name]["status"] = ["UPDATE_IN_PROGRESS", "UPDATE_COMPLETE"]
            return 200, f"<UpdateStackResponse {ns}/>", "text/xml"
        if a == "DeleteStack":
            self.stacks[name]["status"] = ["DELETE_IN_PROGRESS", None]
            return 200, f"<DeleteStackResponse {ns}/>", "text/xml"
        if a == "DescribeStacks":
            members = ""
            for n, s in list(self.stacks.items()):
                if name and n != name:
                    continue
                st = s["status"][0]
                if len(s["status"]) > 1:
                    s["status"].pop(0)
                if st is None:
                    del self.stacks[n]
                    continue
                outs = "<member><OutputKey>MasterAddress</OutputKey><OutputValue>ec2-1.compute.amazonaws.com</OutputValue></member>" \
                    if st.endswith("COMPLETE") else ""
                members += (f"<member><StackName>{n}</StackName><StackStatus>{st}</StackStatus><Outputs>{outs}</Outputs>"
                            f"<Tags><member><Key>{aws.TAG_KEY}</Key><Value>{n}</Value></member></Tags></member>")
            if name and not members:
                return 400, f"<ErrorResponse><Error><Message>Stack with id {name} does not exist</Message></Error></ErrorResponse>", "text/xml"
            return 200, f"<DescribeStacksResponse {ns}><DescribeStacksResult><Stacks>{members}</Stacks></DescribeStacksResult></DescribeStacksResponse>", "text/xml"
        return 400, "<ErrorResponse/>", "text/xml"


def _aws_args(**kw):
    a = dict(region="us-west-2", deployment_type="vpc", cluster_id="mi355x", keypair="kp", image_id="ami-1",
             gpu_agent_instance_type="gpu.8x", master_instance_type="m7i.2xlarge", inbound_cidr="10.0.0.0/8",
             max_dynamic_agents=2, min_dynamic_agents=0, slots_per_instance=8, max_idle_agent_period="5m",
             scheduler_type="fair_share", preemption_enabled=True, poll_interval=0.01, no_wait=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_aws_up_list_down_against_fake_cloudformation():
    cf_fake = FakeCloudFormation()
    ec2 = FakeEC2()
    try:
        cf = aws.CloudFormation("us-west-2", "AKIDEXAMPLE", "secret", endpoint=cf_fake.url)
        logs = []
        s = aws.up(_aws_args(), cf=cf, log=logs.append)
        assert s["status"] == "CREATE_COMPLETE" and s["outputs"]["MasterAddress"].startswith("ec2-")
        create = cf_fake.stacks["mi355x"]["params"]
        params = {create[k]: create[k.replace("ParameterKey", "ParameterValue")]
                  for k in create if k.endswith("ParameterKey")}
        assert params["GpuAgentInstanceType"] == "gpu.8x" and params["SchedulerType"] == "fair_share"
        assert create["Capabilities.member.1"] == "CAPABILITY_IAM"
        _check_refs(json.loads(create["TemplateBody"]))
        assert any("master: http://ec2-" in m for m in logs)
        # a second up is an update
        aws.up(_aws_args(), cf=cf, log=logs.append)
        assert any(c["Action"] == "UpdateStack" for c in cf_fake.calls)
        assert [x["name"] for x in aws.list_clusters(_aws_args(), cf=cf)] == ["mi355x"]
        # down terminates provisioner-launched agents by tag, then deletes the stack
        from determined_clone_amd.master.provisioner import AWSProvider

        prov = AWSProvider("default", {"endpoint_url": ec2.url, "access_key": "AKIDEXAMPLE", "secret_key": "s",
                                       "tag_key": aws.TAG_KEY, "tag_value": "mi355x"}, "http://10.0.0.5:8080")
        prov.launch(2)
        aws.down(_aws_args(), cf=cf, log=logs.append, ec2=prov)
        assert all(i["state"] == "terminated" for i in ec2.instances.values())
        assert "mi355x" not in cf_fake.stacks
        aws.down(_aws_args(), cf=cf, log=logs.append, ec2=prov)  # idempotent
        assert logs[-1] == "no stack mi355x"
    finally:
        cf_fake.srv.stop()
        ec2.stop()


def test_aws_provider_uses_instance_profile_credentials():
    """No static keys: the provisioner signs with IMDSv2 instance-profile credentials."""
    ec2 = FakeEC2(access_key="ASIAROLE")
    seen = []

    def imds(method, path, body, headers):
        seen.append((method, path))
        if method == "PUT" and path == "/latest/api/token":
            return 200, "tok", "text/plain"
        if headers.get("X-aws-ec2-metadata-token") != "tok":
            return 401, "", "text/plain"
        if path == "/latest/meta-data/iam/security-credentials/":
            return 200, "det-master-role\n", "text/plain"
        if path == "/latest/meta-data/iam/security-credentials/det-master-role":
            return 200, json.dumps({"AccessKeyId": "ASIAROLE", "SecretAccessKey": "s", "Token": "t",
                                    "Expiration": "2099-01-01T00:00:00Z"}), "application/json"
        return 404, "", "text/plain"

    md = _Srv(imds)
    old = {k: os.environ.pop(k, None) for k in ("AWS_ACCESS_KEY_ID", "AWS_SECRET_ACCESS_KEY", "AWS_SESSION_TOKEN")}
    try:
        from determined_clone_amd.master.provisioner import AWSProvider

        p = AWSProvider("default", {"endpoint_url": ec2.url, "imds_endpoint": md.url}, "http://m:8080")
        assert p.list() == [] and p.token == "t"
        n = len(seen)
        p.list()
        assert len(seen) == n  # cached until close to expiry
    finally:
        for k, v in old.items():
            if v is not None:
                os.environ[k] = v
        md.stop()
        ec2.stop()


# ============================================================================ GCP
def _gcp_args(tmp_path, **kw):
    a = dict(cluster_id="c1", project_id="proj", region="us-central1", zone=None, environment_image="img-rocm",
             gpu_agent_instance_type="a3-gpu-8", gpu_type=None, gpu_num=8, master_instance_type="n2-standard-4",
             inbound_cidr="0.0.0.0/0", port=8080, disk_size=500, preemptible=False, min_dynamic_agents=0,
             max_dynamic_agents=3, max_idle_agent_period="10m", scheduler_type="priority",
             tf_state_gcs_bucket_name=None, local_state_path=str(tmp_path / "state"), dry_run=False)
    a.update(kw)
    return argparse.Namespace(**a)


def test_gcp_terraform_config_consistent(tmp_path):
    cfg = gcp.terraform_config(gcp.values(_gcp_args(tmp_path, tf_state_gcs_bucket_name="tfstate")))
    res = cfg["resource"]
    text = json.dumps(cfg)
    # every ${type.name.attr} interpolation names a declared resource
    for ref in re.findall(r"(?<!\$)\$\{([a-z_]+)\.([a-z_0-9]+)\.", text):
        assert ref[1] in res.get(ref[0], {}), ref
    assert cfg["terraform"]["backend"]["gcs"]["bucket"] == "tfstate"
    for d in res["google_compute_instance"]["master"]["depends_on"]:
        t, n = d.split(".")
        assert n in res[t]
    script = res["google_compute_instance"]["master"]["metadata_startup_script"]
    body = script.split("master.yaml <<EOF\n", 1)[1].split("\nEOF", 1)[0]
    master = yaml.safe_load(body.replace("$${IP}", "10.20.0.2").replace("${google_service_account.det.email}", "sa@x"))
    prov = master["resource_pools"][0]["provider"]
    assert prov["type"] == "gcp" and prov["service_account"]["email"] == "sa@x"
    assert prov["instance_type"]["machine_type"] == "a3-gpu-8" and prov["slots_per_instance"] == 8
    assert master["checkpoint_storage"] == {"type": "gcs", "bucket": "proj-det-c1-checkpoints"}
    assert master["external_url"] == "http://10.20.0.2:8080"
    with pytest.raises(ValueError):
        gcp.values(_gcp_args(tmp_path, environment_image=None))


def test_gcp_up_down_with_fake_terraform(tmp_path):
    log = tmp_path / "tf.log"
    tf = _script(tmp_path / "terraform", f"""echo "$PWD $*" >> {log}
if [ "$1" = output ]; then echo '{{"master_url": {{"value": "http://35.0.0.1:8080"}}}}'; fi
""")
    args = _gcp_args(tmp_path)
    assert gcp.up(_gcp_args(tmp_path, dry_run=True), log=lambda m: None) is None
    assert not log.exists()
    out = gcp.up(args, log=lambda m: None, tf_bin=tf)
    assert out == {"master_url": "http://35.0.0.1:8080"}
    d = gcp.state_dir(args)
    assert log.read_text().splitlines()[:2] == [f"{d} init -input=false", f"{d} apply -input=false -auto-approve"]
    assert gcp.list_clusters(args) == ["c1"]
    gce = FakeGCE()
    try:
        from determined_clone_amd.master.provisioner import GCPProvider

        prov = GCPProvider("default", {"project": "proj", "zone": "us-central1-a", "endpoint_url": gce.url,
                                       "token": "gce-token", "labels": {gcp.LABEL: "c1"}}, "http://10.20.0.2:8080")
        prov.launch(2)
        body = gce.bodies[0]["instanceProperties"]
        assert body["networkInterfaces"][0]["accessConfigs"][0]["type"] == "ONE_TO_ONE_NAT"
        lister = GCPProvider("default", {"project": "proj", "zone": "us-central1-a", "endpoint_url": gce.url,
                                         "token": "gce-token"}, "http://10.20.0.2:8080")
        # the fake matches an instance only when the filter names all its determined-* labels
        lister.labels = dict(prov.labels, **{gcp.LABEL: "c1"})
        gcp.down(args, log=lambda m: None, tf_bin=tf, gce=lister)
        assert all(i["status"] == "DELETED" for i in gce.instances.values())
    finally:
        gce.stop()
    lines = log.read_text().splitlines()
    assert lines[-2:] == [f"{d} state rm google_storage_bucket.checkpoints", f"{d} destroy -input=false -auto-approve"]


# ============================================================================ GKE
def test_gke_plan_and_up(tmp_path):
    args = argparse.Namespace(cluster_id="g1", region=None, zone="us-central1-a", master_machine_type="n2-standard-4",
                              agent_machine_type="gpu-node", gpu_type="amd-mi355x", gpus_per_node=8, max_gpu_nodes=2,
                              gpu_node_pool_name="accel", slot_resource="amd.com/gpu", gcs_bucket_name=None,
                              no_managed_bucket=False, namespace="determined", image="reg/det:2", dry_run=False)
    cmds = gke.plan(args)
    assert cmds[0][:4] == ["gcloud", "storage", "buckets", "create"] and cmds[0][5:] == ["--location", "us-central1"]
    pool = next(c for c in cmds if c[2] == "node-pools")
    assert "type=amd-mi355x,count=8" in pool and pool[pool.index("--max-nodes") + 1] == "2"
    ran = []
    kb = _script(tmp_path / "kubectl", "if [ \"$3\" = get ]; then echo '{}'; else cat > /dev/null; fi\n")
    gke.up(args, log=lambda m: None, runner=lambda c, check: ran.append(c), kubectl_bin=kb)
    assert ran == cmds
    v = gke.install_values(args)
    assert v["checkpoint_storage"] == {"type": "gcs", "bucket": "det-g1-checkpoints"} and v["max_slots_per_pod"] == 8
    printed = []
    gke.up(argparse.Namespace(**dict(vars(args), dry_run=True)), log=printed.append)
    assert printed[0].startswith("gcloud storage buckets create")
    gke.down(args, log=lambda m: None, runner=lambda c, check: ran.append(c))
    assert ran[-1][:4] == ["gcloud", "container", "clusters", "delete"]


# ============================================================================ CLI / health
def test_deploy_cli_commands(capsys):
    p = build_parser()
    a = p.parse_args(["deploy", "aws", "print-template", "--deployment-type", "vpc"])
    a.func(a)
    tpl = json.loads(capsys.readouterr().out)
    assert "PublicSubnet" in tpl["Resources"]
    a = p.parse_args(["deploy", "k8s", "render", "--namespace", "abc", "--service-type", "NodePort"])
    a.func(a)
    docs = list(yaml.safe_load_all(capsys.readouterr().out))
    assert next(d for d in docs if d["kind"] == "Service")["spec"]["type"] == "NodePort"
    a = p.parse_args(["deploy", "gcp", "up", "--cluster-id", "c", "--project-id", "p", "--environment-image", "i",
                      "--gpu-agent-instance-type", "t", "--dry-run", "--local-state-path", "/tmp/det-deploy-test"])
    assert a.dry_run and a.func.__name__ == "_gcp"


def test_wait_for_master(tmp_path):
    from determined_clone_amd.master.core import Master
    from determined_clone_amd.master.server import MasterServer

    srv = MasterServer(Master(str(tmp_path / "m.db")), port=0).start()
    try:
        info = wait_for_master(f"http://127.0.0.1:{srv.port}", timeout=10)
        assert info["product"] == "determined_clone_amd"
    finally:
        srv.stop()
    with pytest.raises(TimeoutError):
        wait_for_master("http://127.0.0.1:1", timeout=0.5, interval=0.1)
