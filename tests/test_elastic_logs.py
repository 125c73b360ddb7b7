"""Elasticsearch task-log backend (reference: `master/internal/elastic/elastic_task_logs.go`,
master.yaml ``logging.type: elastic``) against an in-process fake of the ``_bulk`` / ``_search``
REST subset it uses; the master's log endpoints behave as with the sqlite store."""
import base64
import json
import threading
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import pytest

from determined_clone_amd.master.core import Master
from determined_clone_amd.master.logstore import ElasticLogStore, SqliteLogStore, make_log_store


class FakeES:
    def __init__(self, user="elastic", password="pw"):
        self.docs = {}  # index -> [doc]
        self.auth = "Basic " + base64.b64encode(f"{user}:{password}".encode()).decode()
        fake = self

        class H(BaseHTTPRequestHandler):
            def log_message(self, *a):
                pass

            def do_POST(self):
                n = int(self.headers.get("Content-Length") or 0)
                body = self.rfile.read(n).decode()
                if self.headers.get("Authorization") != fake.auth:
                    return self._send(401, {"error": "auth"})
                path = self.path.split("?")[0]
                if path == "/_bulk":
                    lines = [json.loads(x) for x in body.splitlines() if x.strip()]
                    items = []
                    for meta, doc in zip(lines[::2], lines[1::2]):
                        fake.docs.setdefault(meta["index"]["_index"], []).append(doc)
                        items.append({"index": {"status": 201}})
                    return self._send(200, {"errors": False, "items": items})
                if path.endswith("/_search"):
                    return self._send(200, fake.search(path.split("/")[1], json.loads(body)))
                self._send(404, {"error": "no route"})

            def _send(self, code, obj):
                data = json.dumps(obj).encode()
                self.send_response(code)
                self.send_header("Content-Type", "application/json")
                self.send_header("Content-Length", str(len(data)))
                self.end_headers()
                self.wfile.write(data)

        self.httpd = ThreadingHTTPServer(("127.0.0.1", 0), H)
        self.port = self.httpd.server_address[1]
        threading.Thread(target=self.httpd.serve_forever, daemon=True).start()

    def search(self, pattern, q):
        prefix = pattern.rstrip("*")
        docs = [d for idx, ds in self.docs.items() if idx.startswith(prefix) for d in ds]
        for f in q["query"]["bool"]["filter"]:
            if "term" in f:
                (k, v), = f["term"].items()
                docs = [d for d in docs if d.get(k) == v]
            if "range" in f:
                (k, r), = f["range"].items()
                docs = [d for d in docs if d.get(k, 0) > r["gt"]]
        out = {"hits": {"hits": []}}
        if q.get("aggs"):
            out["aggregations"] = {k: {"buckets": [{"key": v} for v in sorted({d[k] for d in docs if d.get(k) is not None}, key=str)]}
                                   for k in q["aggs"]}
        docs.sort(key=lambda d: d["id"])
        out["hits"]["hits"] = [{"_source": d} for d in docs[: q.get("size", 10)]]
        return out

    def stop(self):
        self.httpd.shutdown()
        self.httpd.server_close()


@pytest.fixture()
def es():
    f = FakeES()
    yield f
    f.stop()


def _log(i, task="t1", rank=0):
    return {"task_id": task, "allocation_id": task + ".a", "agent_id": "node-0", "rank_id": rank,
            "log": f"line {i}\n", "timestamp": 1760000000.0 + i}


def test_master_logs_through_elastic(es, tmp_path):
    cfg = {"type": "elastic", "host": "127.0.0.1", "port": es.port,
           "security": {"username": "elastic", "password": "pw"}}
    m = Master(str(tmp_path / "m.db"), logging_config=cfg)
    assert isinstance(m.logs, ElasticLogStore)
    m.post_logs([_log(i, rank=i % 2) for i in range(5)] + [_log(9, task="other")])
    assert list(es.docs) == ["determined-tasklogs-2025.10.09"]
    rows = m.task_logs("t1")
    assert [r["log"] for r in rows] == [f"line {i}\n" for i in range(5)]
    ids = [r["id"] for r in rows]
    assert ids == sorted(ids) and len(set(ids)) == 5
    assert [r["log"] for r in m.task_logs("t1", after_id=ids[2])] == ["line 3\n", "line 4\n"]
    f = m.logs.fields("t1")
    assert f["rank_id"] == [0, 1] and f["agent_id"] == ["node-0"]
    # ids continue across master restarts (the counter is persisted), so follow cursors stay valid
    m2 = Master(str(tmp_path / "m.db"), logging_config=cfg)
    m2.post_logs([_log(10)])
    assert m2.task_logs("t1", after_id=ids[-1])[0]["id"] > ids[-1]


def test_store_selection_and_errors(es, tmp_path):
    m = Master(str(tmp_path / "m.db"))
    assert isinstance(m.logs, SqliteLogStore)
    with pytest.raises(ValueError):
        make_log_store({"type": "splunk"}, m.db)
    bad = ElasticLogStore({"host": "127.0.0.1", "port": es.port}, m.db)  # no credentials
    with pytest.raises(RuntimeError, match="401"):
        bad.append([dict(_log(1), id=None)])
