"""``det deploy aws``: a cluster on EC2 as one CloudFormation stack (reference:
`deploy/aws/cli.py`, `deploy/aws/aws.py` (boto3 stack create/update/delete),
`deploy/aws/deployment_types/*.py` and the CloudFormation templates under `deploy/aws/templates/`).

Built without boto3: ``template(params)`` produces the stack template as a Python dict and
``CloudFormation`` speaks the CloudFormation query API signed with SigV4 (the same signer the
S3 checkpoint store and the EC2 provisioner use).

The stack (deployment types ``simple`` = default VPC, ``vpc`` = a new VPC + public subnet):

* checkpoint bucket (retained on ``down``),
* master / agent security groups (master API from ``--inbound-cidr``; agents reach the master and
  each other on every port -- RCCL rendezvous + data traffic between nodes),
* master IAM role (EC2 launch/terminate/describe/tag, ``iam:PassRole`` for the agent role, bucket
  access) and agent IAM role (bucket access), as instance profiles,
* the master instance, whose user data writes ``master.yaml`` -- S3 checkpoints and a resource pool
  whose EC2 provisioner launches GPU agents (8 slots per instance by default: one MI355X node) --
  and starts the master.

The provisioner and the S3 store pick up the instance-profile credentials from IMDSv2, so no keys
are baked into the stack."""
import hashlib
import json
import time
import urllib.parse
import xml.etree.ElementTree as ET
from typing import Any, Callable, Dict, List, Optional

import requests

from determined_clone_amd.common.storage._cloud import sigv4_headers

TAG_KEY = "determined-clone-amd-cluster"
DEPLOYMENT_TYPES = ("simple", "vpc")
TERMINAL_OK = {"CREATE_COMPLETE", "UPDATE_COMPLETE", "DELETE_COMPLETE"}
TERMINAL_BAD = {"CREATE_FAILED", "ROLLBACK_COMPLETE", "ROLLBACK_FAILED", "DELETE_FAILED",
                "UPDATE_ROLLBACK_COMPLETE", "UPDATE_ROLLBACK_FAILED", "UPDATE_FAILED"}

PARAMETERS: Dict[str, Dict[str, Any]] = {
    "Keypair": {"Type": "AWS::EC2::KeyPair::KeyName", "Description": "SSH key pair for the instances"},
    "ImageId": {"Type": "AWS::EC2::Image::Id",
                "Description": "AMI with ROCm 7 + this framework installed (master and agents)"},
    "MasterInstanceType": {"Type": "String", "Default": "m7i.2xlarge"},
    "GpuAgentInstanceType": {"Type": "String",
                             "Description": "instance type of the GPU agents (8x MI355X per instance)"},
    "SlotsPerInstance": {"Type": "Number", "Default": 8},
    "InboundCIDR": {"Type": "String", "Default": "0.0.0.0/0"},
    "MasterPort": {"Type": "Number", "Default": 8080},
    "MinDynamicAgents": {"Type": "Number", "Default": 0},
    "MaxDynamicAgents": {"Type": "Number", "Default": 4},
    "MaxIdleAgentPeriod": {"Type": "String", "Default": "10m"},
    "MaxAgentStartingPeriod": {"Type": "String", "Default": "20m"},
    "AgentRootVolumeSize": {"Type": "Number", "Default": 500},
    "SchedulerType": {"Type": "String", "Default": "priority", "AllowedValues": ["priority", "fair_share", "round_robin"]},
    "PreemptionEnabled": {"Type": "String", "Default": "true", "AllowedValues": ["true", "false"]},
    "Version": {"Type": "String", "Default": "latest"},
}


def _user_data(vpc: bool) -> Dict[str, Any]:
    """Master boot script (``Fn::Sub``): write master.yaml, start the master under systemd."""
    subnet = "\n        subnet_id: ${PublicSubnet}" if vpc else ""
    script = """#!/bin/bash
set -ex
mkdir -p /etc/determined /var/lib/determined
TOKEN=$(curl -sX PUT http://169.254.169.254/latest/api/token -H 'X-aws-ec2-metadata-token-ttl-seconds: 300')
IP=$(curl -s -H "X-aws-ec2-metadata-token: $TOKEN" http://169.254.169.254/latest/meta-data/local-ipv4)
cat > /etc/determined/master.yaml <<EOF
host: 0.0.0.0
port: ${MasterPort}
external_url: http://$IP:${MasterPort}
cluster_name: ${AWS::StackName}
checkpoint_storage:
  type: s3
  bucket: ${CheckpointBucket}
  region: ${AWS::Region}
resource_manager:
  type: agent
  scheduler:
    type: ${SchedulerType}
    preemption: ${PreemptionEnabled}
resource_pools:
  - pool_name: default
    provider:
      type: aws
      region: ${AWS::Region}
      image_id: ${ImageId}
      instance_type: ${GpuAgentInstanceType}
      slots_per_instance: ${SlotsPerInstance}
      min_instances: ${MinDynamicAgents}
      max_instances: ${MaxDynamicAgents}
      max_idle_agent_period: ${MaxIdleAgentPeriod}
      max_agent_starting_period: ${MaxAgentStartingPeriod}
      root_volume_size: ${AgentRootVolumeSize}
      ssh_key_name: ${Keypair}
      iam_instance_profile_arn: ${AgentInstanceProfile.Arn}
      tag_key: """ + TAG_KEY + """
      tag_value: ${AWS::StackName}
      network_interface:
        security_group_id: ${AgentSecurityGroup.GroupId}""" + subnet + """
EOF
cat > /etc/systemd/system/determined-master.service <<EOF
[Unit]
Description=determined_clone_amd master
After=network-online.target
[Service]
Environment=HSA_ENABLE_IPC_MODE_LEGACY=0
ExecStart=/usr/bin/python3 -m determined_clone_amd.master --config-file /etc/determined/master.yaml --db /var/lib/determined/master.db
Restart=always
[Install]
WantedBy=multi-user.target
EOF
systemctl daemon-reload
systemctl enable --now determined-master
"""
    return {"Fn::Base64": {"Fn::Sub": script}}


def template(deployment_type: str = "simple") -> Dict[str, Any]:
    if deployment_type not in DEPLOYMENT_TYPES:
        raise ValueError(f"deployment type must be one of {DEPLOYMENT_TYPES}")
    vpc = deployment_type == "vpc"
    ref = lambda n: {"Ref": n}  # noqa: E731
    gid = lambda n: {"Fn::GetAtt": [n, "GroupId"]}  # noqa: E731
    res: Dict[str, Any] = {
        "CheckpointBucket": {"Type": "AWS::S3::Bucket", "DeletionPolicy": "Retain",
                             "Properties": {"Tags": [{"Key": TAG_KEY, "Value": {"Ref": "AWS::StackName"}}]}},
        "MasterSecurityGroup": {"Type": "AWS::EC2::SecurityGroup", "Properties": {
            "GroupDescription": "determined master",
            "SecurityGroupIngress": [
                {"IpProtocol": "tcp", "FromPort": ref("MasterPort"), "ToPort": ref("MasterPort"), "CidrIp": ref("InboundCIDR")},
                {"IpProtocol": "tcp", "FromPort": 22, "ToPort": 22, "CidrIp": ref("InboundCIDR")}]}},
        "AgentSecurityGroup": {"Type": "AWS::EC2::SecurityGroup", "Properties": {
            "GroupDescription": "determined agents",
            "SecurityGroupIngress": [{"IpProtocol": "tcp", "FromPort": 22, "ToPort": 22, "CidrIp": ref("InboundCIDR")}]}},
        # agents -> master API; master -> agents (task proxies); agent <-> agent (RCCL, rendezvous)
        "AgentToMaster": {"Type": "AWS::EC2::SecurityGroupIngress", "Properties": {
            "GroupId": gid("MasterSecurityGroup"), "IpProtocol": "-1", "SourceSecurityGroupId": gid("AgentSecurityGroup")}},
        "MasterToAgent": {"Type": "AWS::EC2::SecurityGroupIngress", "Properties": {
            "GroupId": gid("AgentSecurityGroup"), "IpProtocol": "-1", "SourceSecurityGroupId": gid("MasterSecurityGroup")}},
        "AgentToAgent": {"Type": "AWS::EC2::SecurityGroupIngress", "Properties": {
            "GroupId": gid("AgentSecurityGroup"), "IpProtocol": "-1", "SourceSecurityGroupId": gid("AgentSecurityGroup")}},
        "AgentRole": {"Type": "AWS::IAM::Role", "Properties": {
            "AssumeRolePolicyDocument": _assume_ec2(),
            "Policies": [{"PolicyName": "checkpoints", "PolicyDocument": _bucket_policy()}]}},
        "AgentInstanceProfile": {"Type": "AWS::IAM::InstanceProfile", "Properties": {"Roles": [ref("AgentRole")]}},
        "MasterRole": {"Type": "AWS::IAM::Role", "Properties": {
            "AssumeRolePolicyDocument": _assume_ec2(),
            "Policies": [
                {"PolicyName": "checkpoints", "PolicyDocument": _bucket_policy()},
                {"PolicyName": "provisioner", "PolicyDocument": {"Version": "2012-10-17", "Statement": [
                    {"Effect": "Allow", "Action": ["ec2:DescribeInstances", "ec2:RunInstances", "ec2:CreateTags",
                                                   "ec2:TerminateInstances", "ec2:DescribeImages"], "Resource": "*"},
                    {"Effect": "Allow", "Action": "iam:PassRole", "Resource": {"Fn::GetAtt": ["AgentRole", "Arn"]}}]}}]}},
        "MasterInstanceProfile": {"Type": "AWS::IAM::InstanceProfile", "Properties": {"Roles": [ref("MasterRole")]}},
        "MasterInstance": {"Type": "AWS::EC2::Instance", "Properties": {
            "ImageId": ref("ImageId"), "InstanceType": ref("MasterInstanceType"), "KeyName": ref("Keypair"),
            "IamInstanceProfile": ref("MasterInstanceProfile"),
            "BlockDeviceMappings": [{"DeviceName": "/dev/sda1", "Ebs": {"VolumeSize": 200, "VolumeType": "gp3"}}],
            "MetadataOptions": {"HttpTokens": "required", "HttpPutResponseHopLimit": 2},
            "Tags": [{"Key": "Name", "Value": {"Fn::Sub": "det-master-${AWS::StackName}"}},
                     {"Key": TAG_KEY, "Value": {"Ref": "AWS::StackName"}}],
            "UserData": _user_data(vpc)}},
    }
    if vpc:
        res.update({
            "VPC": {"Type": "AWS::EC2::VPC", "Properties": {"CidrBlock": "10.0.0.0/16", "EnableDnsHostnames": True,
                                                            "EnableDnsSupport": True}},
            "InternetGateway": {"Type": "AWS::EC2::InternetGateway"},
            "GatewayAttachment": {"Type": "AWS::EC2::VPCGatewayAttachment",
                                  "Properties": {"VpcId": ref("VPC"), "InternetGatewayId": ref("InternetGateway")}},
            "PublicSubnet": {"Type": "AWS::EC2::Subnet", "Properties": {
                "VpcId": ref("VPC"), "CidrBlock": "10.0.0.0/20", "MapPublicIpOnLaunch": True,
                "AvailabilityZone": {"Fn::Select": [0, {"Fn::GetAZs": ""}]}}},
            "RouteTable": {"Type": "AWS::EC2::RouteTable", "Properties": {"VpcId": ref("VPC")}},
            "DefaultRoute": {"Type": "AWS::EC2::Route", "DependsOn": "GatewayAttachment", "Properties": {
                "RouteTableId": ref("RouteTable"), "DestinationCidrBlock": "0.0.0.0/0", "GatewayId": ref("InternetGateway")}},
            "SubnetRoutes": {"Type": "AWS::EC2::SubnetRouteTableAssociation",
                             "Properties": {"SubnetId": ref("PublicSubnet"), "RouteTableId": ref("RouteTable")}},
        })
        for sg in ("MasterSecurityGroup", "AgentSecurityGroup"):
            res[sg]["Properties"]["VpcId"] = ref("VPC")
        res["MasterInstance"]["Properties"]["SubnetId"] = ref("PublicSubnet")
        res["MasterInstance"]["Properties"]["SecurityGroupIds"] = [gid("MasterSecurityGroup")]
        res["MasterInstance"]["DependsOn"] = "DefaultRoute"
    else:
        res["MasterInstance"]["Properties"]["SecurityGroups"] = [ref("MasterSecurityGroup")]
    return {
        "AWSTemplateFormatVersion": "2010-09-09",
        "Description": f"determined_clone_amd cluster ({deployment_type})",
        "Parameters": PARAMETERS,
        "Resources": res,
        "Outputs": {
            "MasterAddress": {"Value": {"Fn::GetAtt": ["MasterInstance", "PublicDnsName"]}},
            "MasterPrivateIp": {"Value": {"Fn::GetAtt": ["MasterInstance", "PrivateIp"]}},
            "MasterPort": {"Value": ref("MasterPort")},
            "CheckpointBucket": {"Value": ref("CheckpointBucket")},
        },
    }


def _assume_ec2() -> Dict[str, Any]:
    return {"Version": "2012-10-17", "Statement": [
        {"Effect": "Allow", "Principal": {"Service": "ec2.amazonaws.com"}, "Action": "sts:AssumeRole"}]}


def _bucket_policy() -> Dict[str, Any]:
    arn = {"Fn::GetAtt": ["CheckpointBucket", "Arn"]}
    return {"Version": "2012-10-17", "Statement": [
        {"Effect": "Allow", "Action": ["s3:ListBucket"], "Resource": arn},
        {"Effect": "Allow", "Action": ["s3:GetObject", "s3:PutObject", "s3:DeleteObject"],
         "Resource": {"Fn::Join": ["", [arn, "/*"]]}}]}


# ----------------------------------------------------------------------------------- API client
def _local(tag: str) -> str:
    return tag.split("}", 1)[-1]


def _children(el: Optional[ET.Element], tag: str) -> List[ET.Element]:
    return [] if el is None else [c for c in el if _local(c.tag) == tag]


def _child(el: Optional[ET.Element], tag: str) -> Optional[ET.Element]:
    kids = _children(el, tag)
    return kids[0] if kids else None


def _text(el: Optional[ET.Element], tag: str) -> str:
    c = _child(el, tag)
    return (c.text or "") if c is not None else ""


class CloudFormation:
    """CloudFormation query API (``Version=2010-05-15``), SigV4-signed."""

    def __init__(self, region: str, access_key: str, secret_key: str, token: Optional[str] = None,
                 endpoint: Optional[str] = None, session: Optional[requests.Session] = None) -> None:
        self.region = region
        self.endpoint = endpoint or f"https://cloudformation.{region}.amazonaws.com/"
        self.access_key, self.secret_key, self.token = access_key, secret_key, token
        self.http = session or requests.Session()

    def call(self, action: str, params: Dict[str, str]) -> ET.Element:
        body = urllib.parse.urlencode({"Action": action, "Version": "2010-05-15", **params})
        h = sigv4_headers("POST", self.endpoint, {"content-type": "application/x-www-form-urlencoded; charset=utf-8"},
                          hashlib.sha256(body.encode()).hexdigest(), self.access_key, self.secret_key,
                          self.region, "cloudformation", session_token=self.token)
        r = self.http.post(self.endpoint, data=body, headers=h, timeout=60)
        if r.status_code >= 300:
            msg = r.text
            try:
                err = ET.fromstring(r.content)
                msg = next((e.text for e in err.iter() if _local(e.tag) == "Message"), msg)
            except ET.ParseError:
                pass
            raise RuntimeError(f"CloudFormation {action}: HTTP {r.status_code}: {str(msg)[:400]}")
        return ET.fromstring(r.content)

    def describe(self, stack: Optional[str] = None) -> List[Dict[str, Any]]:
        try:
            root = self.call("DescribeStacks", {"StackName": stack} if stack else {})
        except RuntimeError as e:
            if stack and "does not exist" in str(e):
                return []
            raise
        out = []
        for m in root.iter():
            if _local(m.tag) != "member" or _child(m, "StackStatus") is None:
                continue
            out.append({
                "name": _text(m, "StackName"), "status": _text(m, "StackStatus"),
                "reason": _text(m, "StackStatusReason"),
                "outputs": {_text(o, "OutputKey"): _text(o, "OutputValue") for o in _children(_child(m, "Outputs"), "member")},
                "tags": {_text(t, "Key"): _text(t, "Value") for t in _children(_child(m, "Tags"), "member")},
            })
        return out

    def deploy(self, stack: str, body: str, parameters: Dict[str, str], tags: Dict[str, str]) -> str:
        p: Dict[str, str] = {"StackName": stack, "TemplateBody": body, "Capabilities.member.1": "CAPABILITY_IAM"}
        for i, (k, v) in enumerate(sorted(parameters.items()), 1):
            p[f"Parameters.member.{i}.ParameterKey"] = k
            p[f"Parameters.member.{i}.ParameterValue"] = str(v)
        for i, (k, v) in enumerate(sorted(tags.items()), 1):
            p[f"Tags.member.{i}.Key"] = k
            p[f"Tags.member.{i}.Value"] = v
        if self.describe(stack):
            try:
                self.call("UpdateStack", p)
            except RuntimeError as e:
                if "No updates are to be performed" not in str(e):
                    raise
            return "update"
        self.call("CreateStack", p)
        return "create"

    def delete(self, stack: str) -> None:
        self.call("DeleteStack", {"StackName": stack})

    def wait(self, stack: str, timeout: float = 3600, interval: float = 15.0,
             log: Optional[Callable[[str], None]] = None, gone_ok: bool = False) -> Dict[str, Any]:
        deadline = time.time() + timeout
        last = None
        while True:
            st = self.describe(stack)
            if not st:
                if gone_ok:
                    return {"name": stack, "status": "DELETE_COMPLETE", "outputs": {}}
                raise RuntimeError(f"stack {stack} not found")
            s = st[0]
            if s["status"] != last and log:
                log(f"{stack}: {s['status']}")
            last = s["status"]
            if s["status"] in TERMINAL_OK:
                return s
            if s["status"] in TERMINAL_BAD:
                raise RuntimeError(f"stack {stack}: {s['status']} {s['reason']}")
            if time.time() > deadline:
                raise TimeoutError(f"stack {stack} still {s['status']} after {timeout:.0f}s")
            time.sleep(interval)


# ----------------------------------------------------------------------------------- commands
def stack_parameters(args: Any) -> Dict[str, str]:
    p = {"Keypair": args.keypair, "ImageId": args.image_id, "GpuAgentInstanceType": args.gpu_agent_instance_type,
         "MasterInstanceType": args.master_instance_type, "InboundCIDR": args.inbound_cidr,
         "MaxDynamicAgents": args.max_dynamic_agents, "MinDynamicAgents": args.min_dynamic_agents,
         "SlotsPerInstance": args.slots_per_instance, "MaxIdleAgentPeriod": args.max_idle_agent_period,
         "SchedulerType": args.scheduler_type,
         "PreemptionEnabled": "true" if args.preemption_enabled else "false"}
    return {k: str(v) for k, v in p.items() if v is not None}


def client(args: Any) -> CloudFormation:
    import os

    ak = os.environ.get("AWS_ACCESS_KEY_ID", "")
    sk = os.environ.get("AWS_SECRET_ACCESS_KEY", "")
    if not (ak and sk):
        raise RuntimeError("set AWS_ACCESS_KEY_ID / AWS_SECRET_ACCESS_KEY (and AWS_SESSION_TOKEN) to deploy")
    return CloudFormation(args.region, ak, sk, os.environ.get("AWS_SESSION_TOKEN"),
                          endpoint=getattr(args, "endpoint_url", None))


def up(args: Any, cf: Optional[CloudFormation] = None, log: Callable[[str], None] = print) -> Dict[str, Any]:
    cf = cf or client(args)
    body = json.dumps(template(args.deployment_type))
    op = cf.deploy(args.cluster_id, body, stack_parameters(args), {TAG_KEY: args.cluster_id})
    log(f"{op} stack {args.cluster_id} ({args.deployment_type}) in {args.region}")
    if getattr(args, "no_wait", False):
        return {"name": args.cluster_id, "status": "IN_PROGRESS", "outputs": {}}
    s = cf.wait(args.cluster_id, log=log, interval=getattr(args, "poll_interval", 15.0))
    out = s["outputs"]
    if out.get("MasterAddress"):
        log(f"master: http://{out['MasterAddress']}:{out.get('MasterPort', 8080)}")
    return s


def down(args: Any, cf: Optional[CloudFormation] = None, log: Callable[[str], None] = print,
         ec2: Any = None) -> None:
    cf = cf or client(args)
    if not cf.describe(args.cluster_id):
        log(f"no stack {args.cluster_id}")
        return
    # dynamic agents are launched by the master's provisioner, outside the stack: terminate them
    # by tag first, or they would outlive the cluster
    if ec2 is None:
        from determined_clone_amd.master.provisioner import AWSProvider

        ec2 = AWSProvider("default", {"region": args.region, "tag_key": TAG_KEY, "tag_value": args.cluster_id,
                                      "endpoint_url": getattr(args, "ec2_endpoint_url", None)}, "")
    agents = [i.id for i in ec2.list()]
    if agents:
        ec2.terminate(agents)
        log(f"terminated {len(agents)} agent instance(s)")
    cf.delete(args.cluster_id)
    log(f"deleting stack {args.cluster_id} (the checkpoint bucket is retained)")
    if not getattr(args, "no_wait", False):
        cf.wait(args.cluster_id, log=log, gone_ok=True, interval=getattr(args, "poll_interval", 15.0))


def list_clusters(args: Any, cf: Optional[CloudFormation] = None) -> List[Dict[str, Any]]:
    cf = cf or client(args)
    return [s for s in cf.describe() if TAG_KEY in s["tags"]]
