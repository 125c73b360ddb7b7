"""Webhooks (reference master/internal/webhooks): signed delivery from a persisted queue with
exponential backoff, redelivery after a receiver outage and after a master restart, Slack Block
Kit bodies, TASK_LOG regex triggers firing once per (task, trigger), trigger validation."""
import hashlib
import hmac
import json
import threading
import time
import urllib.error
import urllib.request
from http.server import BaseHTTPRequestHandler, HTTPServer

import pytest

from determined_clone_amd.master.core import Master
from determined_clone_amd.master.server import MasterServer

FAST = {"signing_key": "s3cret", "retry_attempts": 6, "retry_initial_s": 0.05, "retry_max_s": 0.2}


class Receiver:
    """Local webhook endpoint; ``fail`` > 0 answers that many requests with HTTP 503."""

    def __init__(self) -> None:
        self.got, self.fail, self.lock = [], 0, threading.Lock()
        outer = self

        class H(BaseHTTPRequestHandler):
            def do_POST(self):
                body = self.rfile.read(int(self.headers["Content-Length"]))
                with outer.lock:
                    if outer.fail > 0:
                        outer.fail -= 1
                        self.send_response(503)
                        self.end_headers()
                        return
                    outer.got.append(({k.lower(): v for k, v in self.headers.items()}, body))
                self.send_response(200)
                self.end_headers()

            def log_message(self, *a):
                pass

        self.srv = HTTPServer(("127.0.0.1", 0), H)
        self.url = f"http://127.0.0.1:{self.srv.server_port}/hook"
        threading.Thread(target=self.srv.serve_forever, daemon=True).start()

    def wait(self, n: int, timeout: float = 10.0):
        t0 = time.time()
        while time.time() - t0 < timeout:
            with self.lock:
                if len(self.got) >= n:
                    return list(self.got)
            time.sleep(0.02)
        raise AssertionError(f"expected {n} deliveries, got {len(self.got)}")

    def close(self):
        self.srv.shutdown()
        self.srv.server_close()


@pytest.fixture()
def recv():
    r = Receiver()
    yield r
    r.close()


def _api(url, method, path, body=None, token=None):
    req = urllib.request.Request(url + path, method=method, data=json.dumps(body or {}).encode(),
                                 headers={"Content-Type": "application/json",
                                          **({"Authorization": f"Bearer {token}"} if token else {})})
    with urllib.request.urlopen(req) as r:
        return json.loads(r.read())


def _start(tmp_path, cfg=FAST):
    m = Master(str(tmp_path / "m.db"), webhooks_config=cfg)
    srv = MasterServer(m, port=0).start()
    url = f"http://127.0.0.1:{srv.port}"
    tok = _api(url, "POST", "/api/v1/auth/login", {"username": "admin", "password": ""})["token"]
    return m, srv, url, tok


class _Exp:
    def __init__(self, eid, name="exp"):
        self.id = eid
        self.config = {"name": name, "workspace": "ws", "project": "proj",
                       "resources": {"slots_per_trial": 2, "resource_pool": "gpu"}}


def _verify(headers, body, key="s3cret"):
    t = headers["x-determined-ai-signature-timestamp"]  # header names are case-insensitive
    want = hmac.new(key.encode(), f"{t},".encode() + body, hashlib.sha256).hexdigest()
    assert headers["x-determined-ai-signature"] == want
    assert headers["content-type"].startswith("application/json")


def test_signed_state_change_delivery_and_slack_blocks(tmp_path, recv):
    m, srv, url, tok = _start(tmp_path)
    try:
        _api(url, "POST", "/api/v1/webhooks", {"url": recv.url, "webhook_type": "WEBHOOK_TYPE_DEFAULT",
              "triggers": [{"trigger_type": "TRIGGER_TYPE_EXPERIMENT_STATE_CHANGE",
                            "condition": {"state": "STATE_COMPLETED"}}]}, tok)
        _api(url, "POST", "/api/v1/webhooks", {"url": recv.url, "webhook_type": "WEBHOOK_TYPE_SLACK",
              "triggers": [{"trigger_type": "TRIGGER_TYPE_EXPERIMENT_STATE_CHANGE",
                            "condition": {"state": "COMPLETED"}}]}, tok)
        hooks = _api(url, "GET", "/api/v1/webhooks", token=tok)["webhooks"]
        assert hooks[0]["triggers"][0]["trigger_type"] == "TRIGGER_TYPE_EXPERIMENT_STATE_CHANGE"
        m.webhooks.experiment_state_changed(_Exp(7), "ACTIVE")  # no trigger for ACTIVE
        m.webhooks.experiment_state_changed(_Exp(7), "COMPLETED")
        got = recv.wait(2)
        time.sleep(0.2)
        assert len(recv.got) == 2
        bodies = []
        for headers, body in got:
            _verify(headers, body)
            bodies.append(json.loads(body))
        default = next(b for b in bodies if "event_type" in b)
        slack = next(b for b in bodies if "blocks" in b)
        assert default["event_type"] == "EXPERIMENT_STATE_CHANGE"
        assert default["condition"] == {"state": "COMPLETED"}
        exp = default["event_data"]["experiment"]
        assert (exp["id"], exp["state"], exp["slots_per_trial"], exp["resource_pool"], exp["workspace"]) == \
            (7, "COMPLETED", 2, "gpu", "ws")
        assert slack["blocks"][0]["text"]["text"].startswith("Your experiment completed successfully")
        att = slack["attachments"][0]
        assert att["color"] == "#13B670" and att["blocks"][0]["text"]["type"] == "mrkdwn"
        assert {"type": "mrkdwn", "text": "*Workspace*: ws"} in att["blocks"][0]["fields"]
        assert m.webhooks.queued() == 0
        # the test route sends a signed test event
        wid = hooks[0]["id"]
        assert _api(url, "POST", f"/api/v1/webhooks/{wid}/test", token=tok)["completed"]
        h, b = recv.wait(3)[-1]
        _verify(h, b)
        assert json.loads(b)["event_data"] == {"data": "test"}
    finally:
        m.webhooks.close()
        srv.stop()


def test_delivery_retries_through_a_receiver_outage(tmp_path, recv):
    m, srv, url, tok = _start(tmp_path)
    try:
        _api(url, "POST", "/api/v1/webhooks", {"url": recv.url, "triggers": [
            {"trigger_type": "EXPERIMENT_STATE_CHANGE", "condition": {"state": "ERROR"}}]}, tok)
        recv.fail = 3  # three 503s, then up
        m.webhooks.experiment_state_changed(_Exp(3), "ERROR")
        (headers, body), = recv.wait(1)
        _verify(headers, body)
        assert json.loads(body)["event_data"]["experiment"]["state"] == "ERROR"
        assert recv.fail == 0
    finally:
        m.webhooks.close()
        srv.stop()


def test_undelivered_events_survive_a_master_restart(tmp_path, recv):
    # the receiver is down while the first master runs: the event stays in the queue
    down_url = "http://127.0.0.1:9/hook"  # discard port: connection refused
    cfg = dict(FAST, retry_attempts=1000)
    m, srv, url, tok = _start(tmp_path, cfg)
    _api(url, "POST", "/api/v1/webhooks", {"url": down_url, "triggers": [
        {"trigger_type": "EXPERIMENT_STATE_CHANGE", "condition": {"state": "COMPLETED"}}]}, tok)
    m.webhooks.experiment_state_changed(_Exp(11), "COMPLETED")
    time.sleep(0.3)
    m.webhooks.close()  # master stops with the event still undelivered
    srv.stop()
    assert m.webhooks.queued() == 1
    m.db.execute("UPDATE webhooks SET url=?", [recv.url])
    m.db.execute("UPDATE webhook_events_queue SET url=?", [recv.url])  # receiver back at a new address
    m.db.close()
    m2 = Master(str(tmp_path / "m.db"), webhooks_config={k: v for k, v in FAST.items() if k != "signing_key"})
    try:
        (headers, body), = recv.wait(1)
        # the signing key generated-or-configured for the first master is persisted
        _verify(headers, body, key=m2.webhooks.signing_key)
        assert m2.webhooks.signing_key == "s3cret"
        assert json.loads(body)["event_data"]["experiment"]["id"] == 11
        t0 = time.time()
        while m2.webhooks.queued() and time.time() - t0 < 5:
            time.sleep(0.02)
        assert m2.webhooks.queued() == 0
    finally:
        m2.webhooks.close()


def test_task_log_trigger_fires_once_per_task(tmp_path, recv):
    m, srv, url, tok = _start(tmp_path)
    try:
        _api(url, "POST", "/api/v1/webhooks", {"url": recv.url, "triggers": [
            {"trigger_type": "TRIGGER_TYPE_TASK_LOG", "condition": {"regex": "CUDA|HIP error: (.*)"}}]}, tok)
        _api(url, "POST", "/api/v1/task/logs", {"logs": [
            {"task_id": "1.1", "agent_id": "node-3", "log": "step 10 ok"},
            {"task_id": "1.1", "agent_id": "node-3", "log": "HIP error: out of memory"},
            {"task_id": "1.1", "agent_id": "node-3", "log": "HIP error: again"},
            {"task_id": "2.1", "agent_id": "node-4", "log": "HIP error: invalid device"}]}, tok)
        got = recv.wait(2)
        time.sleep(0.3)
        assert len(recv.got) == 2  # once per (task, trigger)
        payloads = sorted((json.loads(b) for _, b in got), key=lambda p: p["event_data"]["task_log"]["task_id"])
        first = payloads[0]
        assert first["event_type"] == "TASK_LOG" and first["condition"] == {"regex": "CUDA|HIP error: (.*)"}
        assert first["event_data"]["task_log"] == {"task_id": "1.1", "node_name": "node-3",
                                                   "triggering_log": "HIP error: out of memory"}
        for h, b in got:
            _verify(h, b)
    finally:
        m.webhooks.close()
        srv.stop()


def test_trigger_validation(tmp_path):
    m, srv, url, tok = _start(tmp_path)
    try:
        for bad in ({"trigger_type": "TRIGGER_TYPE_TASK_LOG", "condition": {"regex": "("}},
                    {"trigger_type": "TRIGGER_TYPE_TASK_LOG", "condition": {"state": "x"}},
                    {"trigger_type": "TRIAL_STATE_CHANGE", "condition": {}}):
            with pytest.raises(urllib.error.HTTPError) as e:
                _api(url, "POST", "/api/v1/webhooks", {"url": "http://x", "triggers": [bad]}, tok)
            assert e.value.code == 400
    finally:
        m.webhooks.close()
        srv.stop()
