"""Task-log storage backends (reference: `master/internal/db/postgres_task_logs.go` and
`master/internal/elastic/elastic_task_logs.go`, selected by master.yaml ``logging.type``).

``default``: the master's sqlite ``task_logs`` table. ``elastic``: an Elasticsearch cluster over
its REST API -- batched ``_bulk`` indexing into daily ``<prefix>-YYYY.MM.DD`` indices, ordered
``_search`` for the log-follow cursor, ``terms`` aggregations for the log-field filters. Log ids
are assigned by the master (a persisted counter), so followers can keep resuming ``after_id``."""
import itertools
import json
import threading
import time
from typing import Any, Dict, List, Optional

import requests

FIELDS = ("agent_id", "container_id", "rank_id", "stdtype", "source", "level", "allocation_id")


def normalize(lg: Dict[str, Any], ts: float) -> Dict[str, Any]:
    return {"task_id": lg.get("task_id"), "allocation_id": lg.get("allocation_id"),
            "agent_id": lg.get("agent_id"), "container_id": lg.get("container_id"),
            "rank_id": lg.get("rank_id"), "timestamp": lg.get("timestamp") or ts,
            "level": lg.get("level", "INFO"), "log": lg.get("log", ""),
            "source": lg.get("source", "task"), "stdtype": lg.get("stdtype", "stdout")}


class SqliteLogStore:
    def __init__(self, db: Any) -> None:
        self.db = db

    def append(self, logs: List[Dict[str, Any]]) -> None:
        for lg in logs:
            self.db.insert("task_logs", lg)

    def after(self, task_id: str, after_id: int = 0, limit: int = 10000) -> List[Dict[str, Any]]:
        return self.db.all("SELECT * FROM task_logs WHERE task_id=? AND id>? ORDER BY id LIMIT ?",
                           [task_id, after_id, limit])

    def fields(self, task_id: str) -> Dict[str, List[Any]]:
        rows = self.db.all("SELECT DISTINCT " + ", ".join(FIELDS) + " FROM task_logs WHERE task_id=?", [task_id])
        return {k: sorted({x[k] for x in rows if x[k] is not None}, key=str) for k in FIELDS}


class ElasticLogStore:
    def __init__(self, cfg: Dict[str, Any], db: Any, session: Optional[requests.Session] = None) -> None:
        scheme = "https" if (cfg.get("security") or {}).get("tls", {}).get("enabled") else "http"
        self.url = cfg.get("url") or f"{scheme}://{cfg.get('host', 'localhost')}:{int(cfg.get('port', 9200))}"
        self.url = self.url.rstrip("/")
        sec = cfg.get("security") or {}
        self.http = session or requests.Session()
        if sec.get("username"):
            self.http.auth = (sec["username"], sec.get("password", ""))
        tls = sec.get("tls") or {}
        if tls.get("certificate"):
            self.http.verify = tls["certificate"]
        elif tls.get("skip_verify"):
            self.http.verify = False
        self.prefix = cfg.get("index_prefix", "determined-tasklogs")
        self.db = db
        self._lock = threading.Lock()
        start = int(db.kv_get("elastic_log_seq") or 0)
        self._ids = itertools.count(start + 1)
        self._last = start

    def _index(self, ts: float) -> str:
        return f"{self.prefix}-{time.strftime('%Y.%m.%d', time.gmtime(ts))}"

    def _post(self, path: str, data: Any, ndjson: bool = False) -> Dict[str, Any]:
        headers = {"Content-Type": "application/x-ndjson" if ndjson else "application/json"}
        r = self.http.post(self.url + path, data=data if ndjson else json.dumps(data), headers=headers, timeout=30)
        if r.status_code >= 300:
            raise RuntimeError(f"elasticsearch {path}: HTTP {r.status_code}: {r.text[:300]}")
        return r.json() if r.content else {}

    def append(self, logs: List[Dict[str, Any]]) -> None:
        if not logs:
            return
        lines = []
        with self._lock:
            for lg in logs:
                doc = dict(lg, id=next(self._ids))
                self._last = doc["id"]
                lines.append(json.dumps({"index": {"_index": self._index(float(doc["timestamp"]))}}))
                lines.append(json.dumps(doc))
            self.db.kv_set("elastic_log_seq", str(self._last))
        out = self._post("/_bulk?refresh=wait_for", "\n".join(lines) + "\n", ndjson=True)
        if out.get("errors"):
            bad = [i for i in out.get("items", []) if (i.get("index") or {}).get("error")]
            raise RuntimeError(f"elasticsearch bulk index: {len(bad)} of {len(logs)} logs rejected")

    def after(self, task_id: str, after_id: int = 0, limit: int = 10000) -> List[Dict[str, Any]]:
        q = {"query": {"bool": {"filter": [{"term": {"task_id": task_id}},
                                           {"range": {"id": {"gt": int(after_id)}}}]}},
             "sort": [{"id": "asc"}], "size": int(limit)}
        hits = self._post(f"/{self.prefix}-*/_search", q).get("hits", {}).get("hits", [])
        return [h["_source"] for h in hits]

    def fields(self, task_id: str) -> Dict[str, List[Any]]:
        q = {"size": 0, "query": {"bool": {"filter": [{"term": {"task_id": task_id}}]}},
             "aggs": {k: {"terms": {"field": k, "size": 1000}} for k in FIELDS}}
        aggs = self._post(f"/{self.prefix}-*/_search", q).get("aggregations", {})
        return {k: sorted((b["key"] for b in (aggs.get(k) or {}).get("buckets", [])), key=str) for k in FIELDS}


def make_log_store(cfg: Optional[Dict[str, Any]], db: Any) -> Any:
    t = (cfg or {}).get("type", "default")
    if t in ("default", "sqlite", None):
        return SqliteLogStore(db)
    if t == "elastic":
        return ElasticLogStore(cfg or {}, db)
    raise ValueError(f"unknown logging.type {t!r} (default | elastic)")
