"""Master observability: Prometheus state / process metrics and the audit log (reference:
`master/internal/prom/det_state_metrics.go`, `master/internal/audit.go`)."""
import json
import logging
import urllib.request

import pytest

from determined_clone_amd.master.core import Allocation, Master
from determined_clone_amd.master.server import MasterServer


@pytest.fixture()
def master(tmp_path):
    m = Master(str(tmp_path / "m.db"))
    srv = MasterServer(m, port=0).start()
    yield m, f"http://127.0.0.1:{srv.port}"
    srv.stop()


def _get(url):
    with urllib.request.urlopen(url) as r:
        return r.headers["Content-Type"], r.read().decode()


def _call(url, method, path, body, token):
    req = urllib.request.Request(url + path, method=method, data=json.dumps(body).encode(),
                                 headers={"Content-Type": "application/json", "Authorization": f"Bearer {token}"})
    with urllib.request.urlopen(req) as r:
        return json.loads(r.read())


def test_state_metrics_join_gpus_to_allocations(master):
    m, url = master
    m.register_agent({"agent_id": "node-0", "slots": [{"id": i, "uuid": f"GPU-{i:04x}", "type": "rocm"} for i in range(8)],
                      "resource_pool": "default"})
    a = Allocation("t9.a", "t9", "COMMAND")
    a.state = "RUNNING"
    a.placements = [{"agent_id": "node-0", "slots": [2, 3]}]
    m.allocations[a.id] = a
    m.rm.agents["node-0"].slot_owner[2] = a.id
    m.rm.agents["node-0"].slot_owner[3] = a.id
    ctype, text = _get(url + "/prom/det-state-metrics")
    assert ctype.startswith("text/plain")
    assert 'det_agent_slots{agent_id="node-0",resource_pool="default",state="used"} 2.0' in text
    assert 'det_agent_slots{agent_id="node-0",resource_pool="default",state="free"} 6.0' in text
    assert 'det_gpu_uuid_allocation{agent_id="node-0",allocation_id="t9.a",gpu_uuid="GPU-0003",slot_id="3",task_id="t9"} 1.0' in text
    assert 'det_allocation_info{allocation_id="t9.a",experiment_id="",task_id="t9",task_type="COMMAND",trial_id=""} 1.0' in text


def test_process_metrics_count_requests(master):
    m, url = master
    _get(url + "/api/v1/master")
    _, text = _get(url + "/debug/prom/metrics")
    assert 'det_api_requests_total{code="200",handler="master_info",method="GET"}' in text
    assert "det_api_request_seconds_bucket" in text


def test_audit_log_records_mutations(master, caplog):
    m, url = master
    tok, _ = m.login("admin", "")
    # a handler on the audit logger itself: independent of propagation / root-level settings other
    # tests in the same worker process may have changed
    records = []

    class _Keep(logging.Handler):
        def emit(self, record):
            records.append(record)

    lg = logging.getLogger("determined_clone_amd.master.audit")
    h = _Keep(level=logging.INFO)
    old_level, old_disabled = lg.level, lg.disabled
    lg.addHandler(h)
    lg.setLevel(logging.INFO)
    lg.disabled = False
    try:
        _call(url, "POST", "/api/v1/workspaces", {"name": "audited"}, tok)
        _get(url + "/api/v1/master")  # reads are not audited
    finally:
        lg.removeHandler(h)
        lg.setLevel(old_level)
        lg.disabled = old_disabled
    recs = [json.loads(r.getMessage()) for r in records]
    assert len(recs) == 1
    assert recs[0]["user"] == "admin" and recs[0]["method"] == "POST"
    assert recs[0]["path"] == "/api/v1/workspaces" and recs[0]["status"] == 200
    assert recs[0]["handler"] == "post_workspace"
