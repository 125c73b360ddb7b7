"""Outgoing webhooks: persisted event queue, signed batch delivery with backoff, Slack blocks,
experiment-state and task-log triggers.

Reference: ``master/internal/webhooks`` --
* ``postgres_webhook.go:220-290``: an event is a row of ``webhook_events_queue`` (URL + payload)
  inserted when a trigger matches; ``TRIGGER_TYPE_TASK_LOG`` triggers keep compiled regexes and
  fire at most once per (task, trigger) (``webhook_task_log_triggers``);
* ``shipper.go:141-232``: worker threads dequeue batches of up to 10 events, deliver each with
  exponential backoff (5xx / connection errors retry, 4xx is permanent), and consume the batch;
  undelivered rows survive a master restart and are shipped at start-up;
* every request is signed: ``X-Determined-AI-Signature`` = hex HMAC-SHA256 of ``"{t},{body}"``
  keyed by ``webhooks.signing_key`` (generated when unset -- here persisted in the master DB so a
  restart keeps it, ``config.go:272-277``), ``X-Determined-AI-Signature-Timestamp`` = t;
* ``api_webhook.go`` / ``postgres_webhook.go:345-560``: DEFAULT payloads are
  ``{event_id, event_type, timestamp, condition, event_data}``; SLACK payloads are Block Kit
  messages (status section + a coloured attachment with Status / Duration / Workspace / Project).
"""
import hashlib
import hmac
import json
import logging
import re
import secrets
import threading
import time
import uuid
from typing import Any, Dict, List, Optional, Tuple

logger = logging.getLogger("determined_clone_amd.master.webhooks")

EXPERIMENT_STATE_CHANGE = "EXPERIMENT_STATE_CHANGE"
METRIC_THRESHOLD_EXCEEDED = "METRIC_THRESHOLD_EXCEEDED"
TASK_LOG = "TASK_LOG"
TRIGGER_TYPES = (EXPERIMENT_STATE_CHANGE, METRIC_THRESHOLD_EXCEEDED, TASK_LOG)
DEFAULT, SLACK = "DEFAULT", "SLACK"

MAX_WORKERS = 3
MAX_BATCH = 10

SCHEMA = """
CREATE TABLE IF NOT EXISTS webhook_events_queue (
  id INTEGER PRIMARY KEY AUTOINCREMENT, url TEXT, payload TEXT, created REAL);
CREATE TABLE IF NOT EXISTS webhook_task_log_triggers (
  task_id TEXT, trigger_key TEXT, PRIMARY KEY (task_id, trigger_key));
"""


def norm_trigger_type(t: Any) -> str:
    """``TRIGGER_TYPE_TASK_LOG`` / ``TASK_LOG`` -> ``TASK_LOG`` (proto enum or DB form)."""
    s = str(t or "").upper()
    return s[len("TRIGGER_TYPE_"):] if s.startswith("TRIGGER_TYPE_") else s


def norm_webhook_type(t: Any) -> str:
    s = str(t or DEFAULT).upper()
    s = s[len("WEBHOOK_TYPE_"):] if s.startswith("WEBHOOK_TYPE_") else s
    return DEFAULT if s in ("", "UNSPECIFIED") else s


def validate_triggers(triggers: Any) -> List[Dict[str, Any]]:
    """Normalised trigger list, or ValueError (reference api_webhook.go PostWebhook checks)."""
    out = []
    for tr in triggers or []:
        if not isinstance(tr, dict):
            raise ValueError(f"webhook trigger must be an object, got {tr!r}")
        tt = norm_trigger_type(tr.get("trigger_type"))
        if tt not in TRIGGER_TYPES:
            raise ValueError(f"unknown webhook trigger type {tr.get('trigger_type')!r}")
        cond = tr.get("condition") or {}
        if tt == TASK_LOG:
            if len(cond) != 1 or "regex" not in cond or not isinstance(cond["regex"], str):
                raise ValueError(f"webhook task log condition must have one string key 'regex', got {cond}")
            try:
                re.compile(cond["regex"])
            except re.error as e:
                raise ValueError(f"invalid task log regex {cond['regex']!r}: {e}") from None
        elif tt == EXPERIMENT_STATE_CHANGE and "state" in cond:
            cond = dict(cond, state=str(cond["state"]).upper().replace("STATE_", "", 1))
        out.append({"trigger_type": tt, "condition": cond})
    return out


def sign(key: str, t: int, body: bytes) -> str:
    return hmac.new(key.encode(), f"{t},".encode() + body, hashlib.sha256).hexdigest()


class WebhookManager:
    """Trigger evaluation + the persisted queue + the delivery workers of one master."""

    def __init__(self, master: Any, config: Optional[Dict[str, Any]] = None) -> None:
        self.master = master
        self.db = master.db
        cfg = dict(config or {})
        self.db._conn.executescript(SCHEMA)
        key = cfg.get("signing_key") or self.db.kv_get("webhooks_signing_key")
        if not key:
            key = secrets.token_hex(6)
        self.db.kv_set("webhooks_signing_key", key)
        self.signing_key = str(key)
        self.base_url = str(cfg.get("base_url") or "").rstrip("/")
        # backoff: the reference retries twice from 1 s up to 1 min; attempts and intervals are
        # configurable here (master.yaml webhooks.retry_attempts / retry_initial_s / retry_max_s)
        self.retry_attempts = int(cfg.get("retry_attempts", 5))
        self.retry_initial = float(cfg.get("retry_initial_s", 1.0))
        self.retry_max = float(cfg.get("retry_max_s", 60.0))
        self.timeout = float(cfg.get("timeout_s", 10.0))
        self._regex_lock = threading.Lock()
        self._regexes: List[Tuple[Any, str, Dict[str, Any]]] = []
        self._cv = threading.Condition()
        self._pending = False
        self._stop = False
        self._inflight: set = set()
        self._workers: List[threading.Thread] = []
        self.reload_triggers()
        for i in range(MAX_WORKERS):
            th = threading.Thread(target=self._work, name=f"webhook-worker-{i}", daemon=True)
            th.start()
            self._workers.append(th)
        self.wake()  # ship whatever a previous master process left in the queue

    # ------------------------------------------------------------------ registry
    def hooks(self) -> List[Dict[str, Any]]:
        from determined_clone_amd.master.db import dec

        return [dict(h, triggers=dec(h["triggers"], []) or []) for h in self.db.all("SELECT * FROM webhooks")]

    def reload_triggers(self) -> None:
        """Recompile the TASK_LOG regexes (after a webhook is added or deleted)."""
        regs = []
        for h in self.hooks():
            for i, tr in enumerate(h["triggers"]):
                if norm_trigger_type(tr.get("trigger_type")) == TASK_LOG:
                    rx = (tr.get("condition") or {}).get("regex")
                    try:
                        regs.append((re.compile(rx), f"{h['id']}:{i}", h))
                    except (re.error, TypeError):
                        logger.warning(f"webhook {h['id']}: bad task log regex {rx!r}")
        with self._regex_lock:
            self._regexes = regs

    # ------------------------------------------------------------------ events
    def _enqueue(self, url: str, payload: Dict[str, Any]) -> None:
        self.db.insert("webhook_events_queue", {"url": url, "payload": json.dumps(payload),
                                                "created": time.time()})
        self.wake()

    def experiment_state_changed(self, exp: Any, state: str) -> None:
        """EXPERIMENT_STATE_CHANGE triggers whose ``condition.state`` equals ``state``."""
        try:
            for h in self.hooks():
                for tr in h["triggers"]:
                    if norm_trigger_type(tr.get("trigger_type")) != EXPERIMENT_STATE_CHANGE:
                        continue
                    want = (tr.get("condition") or {}).get("state")
                    if want is not None and str(want).upper() != state:
                        continue
                    if norm_webhook_type(h["webhook_type"]) == SLACK:
                        payload = self.slack_experiment_payload(exp, state)
                    else:
                        payload = {"event_id": str(uuid.uuid4()), "event_type": EXPERIMENT_STATE_CHANGE,
                                   "timestamp": int(time.time()), "condition": {"state": state},
                                   "event_data": {"experiment": self.experiment_payload(exp, state)}}
                    self._enqueue(h["url"], payload)
        except Exception:  # a webhook must never break the experiment state machine
            logger.exception("webhook experiment event failed")

    def scan_logs(self, logs: List[Dict[str, Any]]) -> None:
        """TASK_LOG triggers: the first log line of a task matching a trigger's regex queues one
        event for that (task, trigger)."""
        with self._regex_lock:
            regs = list(self._regexes)
        if not regs:
            return
        for lg in logs:
            text, task_id = str(lg.get("log", "")), str(lg.get("task_id") or "")
            if not task_id:
                continue
            node = str(lg.get("agent_id") or "")
            for rx, key, h in regs:
                if not rx.search(text):
                    continue
                cur = self.db.execute("INSERT OR IGNORE INTO webhook_task_log_triggers (task_id, trigger_key) "
                                      "VALUES (?, ?)", [task_id, key])
                if cur.rowcount == 0:
                    continue  # this trigger already fired for this task
                if norm_webhook_type(h["webhook_type"]) == SLACK:
                    payload = self.slack_log_payload(task_id, node, rx.pattern, text)
                else:
                    payload = {"event_id": str(uuid.uuid4()), "event_type": TASK_LOG,
                               "timestamp": int(time.time()), "condition": {"regex": rx.pattern},
                               "event_data": {"task_log": {"task_id": task_id, "node_name": node,
                                                           "triggering_log": text}}}
                self._enqueue(h["url"], payload)

    # ------------------------------------------------------------------ payloads
    def experiment_payload(self, exp: Any, state: str) -> Dict[str, Any]:
        row = self.db.one("SELECT start_time, end_time FROM experiments WHERE id=?", [exp.id]) or {}
        start, end = row.get("start_time") or time.time(), row.get("end_time") or time.time()
        cfg = exp.config or {}
        res = cfg.get("resources") or {}
        return {"id": exp.id, "state": state, "name": cfg.get("name") or f"experiment {exp.id}",
                "duration": int(max(0.0, end - start)), "resource_pool": res.get("resource_pool") or "",
                "slots_per_trial": int(res.get("slots_per_trial") or 1),
                "workspace": cfg.get("workspace") or "", "project": cfg.get("project") or ""}

    def slack_experiment_payload(self, exp: Any, state: str) -> Dict[str, Any]:
        p = self.experiment_payload(exp, state)
        ok = state == "COMPLETED"
        title = f"{p['name']} (#{p['id']})"
        link = f"<{self.base_url}/det/experiments/{p['id']}/overview | {title}>" if self.base_url else title
        hours, rem = divmod(p["duration"], 3600)
        fields = [{"type": "mrkdwn", "text": f"*Status*: {'Completed' if ok else 'Errored'}"},
                  {"type": "mrkdwn", "text": f"*Duration*: {hours}h {rem // 60}min"}]
        if p["workspace"]:
            fields.append({"type": "mrkdwn", "text": f"*Workspace*: {p['workspace']}"})
        if p["project"]:
            fields.append({"type": "mrkdwn", "text": f"*Project*: {p['project']}"})
        return {"blocks": [{"type": "section", "text": {
                    "type": "plain_text",
                    "text": "Your experiment completed successfully 🎉" if ok else
                            "Your experiment has stopped with errors"}}],
                "attachments": [{"color": "#13B670" if ok else "#DD5040", "blocks": [
                    {"type": "section", "text": {"type": "mrkdwn", "text": ("✅ " if ok else "❌ ") + link},
                     "fields": fields}]}]}

    def slack_log_payload(self, task_id: str, node: str, regex: str, text: str) -> Dict[str, Any]:
        t = self.db.one("SELECT id, experiment_id FROM trials WHERE task_id=?", [task_id])
        if t is not None:
            msg = (f"Experiment ID `{t['experiment_id']}`, Trial ID `{t['id']}`, running on node `{node}`, "
                   f"reported a log\n```{text}```\nThis log matched the regex\n```{regex}```\n")
            path = f"/det/experiments/{t['experiment_id']}/trials/{t['id']}/logs"
            msg += f"<{self.base_url}{path} | View full logs here>" if self.base_url else f"View full logs at {path}"
        else:
            msg = (f"Task ID `{task_id}`, running on node `{node}`, reported a log\n```{text}```\n"
                   f"This log matched the regex\n```{regex}```\n")
        return {"blocks": [{"type": "section", "text": {"type": "mrkdwn", "text": msg}}]}

    def test_payload(self, webhook_type: str) -> Dict[str, Any]:
        if norm_webhook_type(webhook_type) == SLACK:
            return {"blocks": [{"type": "section", "text": {"type": "plain_text", "text": "test"}}]}
        return {"event_id": str(uuid.uuid4()), "event_type": EXPERIMENT_STATE_CHANGE,
                "timestamp": int(time.time()), "condition": {"state": "COMPLETED"},
                "event_data": {"data": "test"}}

    # ------------------------------------------------------------------ delivery
    def post(self, url: str, payload: Any) -> int:
        """One signed POST; returns the HTTP status (raises on connection errors)."""
        import urllib.error
        import urllib.request

        body = payload if isinstance(payload, bytes) else json.dumps(payload).encode()
        t = int(time.time())
        req = urllib.request.Request(url, data=body, method="POST", headers={
            "Content-Type": "application/json; charset=UTF-8",
            "X-Determined-AI-Signature-Timestamp": str(t),
            "X-Determined-AI-Signature": sign(self.signing_key, t, body)})
        try:
            with urllib.request.urlopen(req, timeout=self.timeout) as resp:
                return int(resp.status)
        except urllib.error.HTTPError as e:
            return int(e.code)

    def deliver(self, url: str, payload: bytes) -> bool:
        """Exponential backoff on connection errors and 5xx; a 4xx is permanent."""
        delay = self.retry_initial
        for attempt in range(self.retry_attempts + 1):
            try:
                code = self.post(url, payload)
                if code < 400:
                    return True
                if code < 500:
                    logger.error(f"webhook {url}: HTTP {code} (not retried)")
                    return False
                err = f"HTTP {code}"
            except Exception as e:  # connection refused, timeout, DNS...
                err = str(e)
            if attempt == self.retry_attempts or self._stop:
                logger.error(f"webhook {url}: giving up after {attempt + 1} attempts: {err}")
                return False
            with self._cv:
                self._cv.wait_for(lambda: self._stop, timeout=delay)
            delay = min(self.retry_max, delay * 2)
        return False

    def wake(self) -> None:
        with self._cv:
            self._pending = True
            self._cv.notify_all()

    def _claim(self) -> List[Dict[str, Any]]:
        with self._cv:
            rows = [r for r in self.db.all("SELECT * FROM webhook_events_queue ORDER BY id LIMIT ?",
                                           [MAX_BATCH + len(self._inflight)])
                    if r["id"] not in self._inflight][:MAX_BATCH]
            self._inflight.update(r["id"] for r in rows)
            if not rows:
                self._pending = False
            return rows

    def _work(self) -> None:
        while True:
            with self._cv:
                self._cv.wait_for(lambda: self._pending or self._stop)
                if self._stop:
                    return
            batch = self._claim()
            if not batch:
                continue
            threads = [threading.Thread(target=self.deliver, args=(r["url"], r["payload"].encode()), daemon=True)
                       for r in batch]
            for th in threads:
                th.start()
            for th in threads:
                th.join()
            with self._cv:
                if self._stop:  # shutting down mid-batch: leave the rows for the next master
                    self._inflight.difference_update(r["id"] for r in batch)
                    return
                # the batch is consumed (delivered, or given up on after the retries)
                for r in batch:
                    self.db.execute("DELETE FROM webhook_events_queue WHERE id=?", [r["id"]])
                self._inflight.difference_update(r["id"] for r in batch)
                self._pending = True

    def queued(self) -> int:
        r = self.db.one("SELECT COUNT(*) AS n FROM webhook_events_queue")
        return int(r["n"]) if r else 0

    def close(self) -> None:
        with self._cv:
            self._stop = True
            self._cv.notify_all()
        for th in self._workers:
            th.join(timeout=5)
