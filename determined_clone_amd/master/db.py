"""Master persistence on SQLite (reference: Postgres via `master/internal/db`, migrations in
`master/static/migrations`). One file, WAL journal, a lock around writes; every table keeps the
JSON blobs the API returns so the master can be restarted and restore experiments."""
import json
import sqlite3
import threading
import time
from typing import Any, Dict, Iterable, List, Optional, Tuple

SCHEMA = """
CREATE TABLE IF NOT EXISTS users (
  id INTEGER PRIMARY KEY AUTOINCREMENT, username TEXT UNIQUE NOT NULL, password_hash TEXT,
  display_name TEXT, admin INTEGER DEFAULT 0, active INTEGER DEFAULT 1, agent_uid INTEGER,
  agent_user TEXT, created REAL, settings TEXT DEFAULT '{}');
CREATE TABLE IF NOT EXISTS sessions (token TEXT PRIMARY KEY, user_id INTEGER, expiry REAL);
CREATE TABLE IF NOT EXISTS groups (id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE);
CREATE TABLE IF NOT EXISTS group_members (group_id INTEGER, user_id INTEGER, PRIMARY KEY(group_id, user_id));
CREATE TABLE IF NOT EXISTS role_assignments (id INTEGER PRIMARY KEY AUTOINCREMENT, role TEXT,
  user_id INTEGER, group_id INTEGER, workspace_id INTEGER);
CREATE TABLE IF NOT EXISTS workspaces (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, user_id INTEGER, archived INTEGER DEFAULT 0,
  pinned INTEGER DEFAULT 0, checkpoint_storage TEXT, default_pool TEXT, created REAL);
CREATE TABLE IF NOT EXISTS projects (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT, workspace_id INTEGER, user_id INTEGER,
  description TEXT DEFAULT '', notes TEXT DEFAULT '[]', archived INTEGER DEFAULT 0, created REAL,
  UNIQUE(workspace_id, name));
CREATE TABLE IF NOT EXISTS experiments (
  id INTEGER PRIMARY KEY AUTOINCREMENT, config TEXT, original_config TEXT, model_definition BLOB,
  state TEXT, progress REAL DEFAULT 0, start_time REAL, end_time REAL, archived INTEGER DEFAULT 0,
  parent_id INTEGER, owner_id INTEGER, project_id INTEGER, job_id TEXT, searcher_snapshot TEXT,
  notes TEXT DEFAULT '', unmanaged INTEGER DEFAULT 0, external_experiment_id TEXT);
CREATE TABLE IF NOT EXISTS trials (
  id INTEGER PRIMARY KEY AUTOINCREMENT, experiment_id INTEGER, request_id TEXT, hparams TEXT,
  state TEXT, start_time REAL, end_time REAL, seed INTEGER, restarts INTEGER DEFAULT 0,
  run_id INTEGER DEFAULT 0, steps_completed INTEGER DEFAULT 0, latest_checkpoint TEXT,
  warm_start_checkpoint TEXT, searcher_state TEXT DEFAULT '{}', summary_metrics TEXT DEFAULT '{}',
  best_validation REAL, latest_validation_steps INTEGER, runner_state TEXT DEFAULT '',
  task_id TEXT, progress REAL DEFAULT 0, tags TEXT DEFAULT '{}', external_trial_id TEXT);
CREATE INDEX IF NOT EXISTS trials_exp ON trials(experiment_id);
CREATE TABLE IF NOT EXISTS metrics (
  id INTEGER PRIMARY KEY AUTOINCREMENT, trial_id INTEGER, trial_run_id INTEGER, grp TEXT,
  steps_completed INTEGER, metrics TEXT, batch_metrics TEXT, end_time REAL, archived INTEGER DEFAULT 0);
CREATE INDEX IF NOT EXISTS metrics_trial ON metrics(trial_id, grp, steps_completed);
CREATE TABLE IF NOT EXISTS checkpoints (
  uuid TEXT PRIMARY KEY, task_id TEXT, allocation_id TEXT, trial_id INTEGER, experiment_id INTEGER,
  report_time REAL, state TEXT, resources TEXT, metadata TEXT, steps_completed INTEGER,
  storage_id INTEGER, size INTEGER DEFAULT 0);
CREATE TABLE IF NOT EXISTS tasks (
  task_id TEXT PRIMARY KEY, task_type TEXT, job_id TEXT, start_time REAL, end_time REAL,
  config TEXT DEFAULT '{}', state TEXT, owner_id INTEGER, workspace_id INTEGER);
CREATE TABLE IF NOT EXISTS allocations (
  allocation_id TEXT PRIMARY KEY, task_id TEXT, slots INTEGER, resource_pool TEXT, start_time REAL,
  end_time REAL, state TEXT, exit_reason TEXT, agent_ids TEXT DEFAULT '[]', proxy TEXT);
CREATE TABLE IF NOT EXISTS task_logs (
  id INTEGER PRIMARY KEY AUTOINCREMENT, task_id TEXT, allocation_id TEXT, agent_id TEXT,
  container_id TEXT, rank_id INTEGER, timestamp REAL, level TEXT, log TEXT, source TEXT, stdtype TEXT);
CREATE INDEX IF NOT EXISTS task_logs_task ON task_logs(task_id, id);
CREATE TABLE IF NOT EXISTS models (
  id INTEGER PRIMARY KEY AUTOINCREMENT, name TEXT UNIQUE, description TEXT DEFAULT '',
  metadata TEXT DEFAULT '{}', labels TEXT DEFAULT '[]', notes TEXT DEFAULT '', archived INTEGER DEFAULT 0,
  user_id INTEGER, workspace_id INTEGER DEFAULT 1, creation_time REAL, last_updated_time REAL);
CREATE TABLE IF NOT EXISTS model_versions (
  id INTEGER PRIMARY KEY AUTOINCREMENT, model_id INTEGER, version INTEGER, checkpoint_uuid TEXT,
  name TEXT, comment TEXT DEFAULT '', notes TEXT DEFAULT '', metadata TEXT DEFAULT '{}',
  labels TEXT DEFAULT '[]', user_id INTEGER, creation_time REAL, last_updated_time REAL,
  UNIQUE(model_id, version));
CREATE TABLE IF NOT EXISTS templates (name TEXT PRIMARY KEY, config TEXT, workspace_id INTEGER DEFAULT 1);
CREATE TABLE IF NOT EXISTS webhooks (
  id INTEGER PRIMARY KEY AUTOINCREMENT, url TEXT, webhook_type TEXT, triggers TEXT, mode TEXT,
  name TEXT, workspace_id INTEGER);
CREATE TABLE IF NOT EXISTS profiler_metrics (
  id INTEGER PRIMARY KEY AUTOINCREMENT, trial_id INTEGER, name TEXT, ts REAL, value TEXT);
CREATE TABLE IF NOT EXISTS kv (key TEXT PRIMARY KEY, value TEXT);
"""


MIGRATIONS = [
    ("experiments", "external_experiment_id", "TEXT"),
    ("trials", "external_trial_id", "TEXT"),
    # profiler series labels (trial/v1 TrialProfilerMetricLabels) and the batch of each reading
    ("profiler_metrics", "agent_id", "TEXT"),
    ("profiler_metrics", "gpu_uuid", "TEXT"),
    ("profiler_metrics", "metric_type", "TEXT"),
    ("profiler_metrics", "batch", "INTEGER"),
]


class DB:
    def __init__(self, path: str = ":memory:") -> None:
        self.path = path
        self._conn = sqlite3.connect(path, check_same_thread=False, isolation_level=None)
        self._conn.row_factory = sqlite3.Row
        self._lock = threading.RLock()
        with self._lock:
            if path != ":memory:":
                self._conn.execute("PRAGMA journal_mode=WAL")
            self._conn.executescript(SCHEMA)
            self._migrate()

    def _migrate(self) -> None:
        """Columns added after a table first shipped (CREATE TABLE IF NOT EXISTS keeps old tables)."""
        for table, col, decl in MIGRATIONS:
            cols = {r[1] for r in self._conn.execute(f"PRAGMA table_info({table})").fetchall()}
            if col not in cols:
                self._conn.execute(f"ALTER TABLE {table} ADD COLUMN {col} {decl}")

    # ------------------------------------------------------------------ primitives
    def execute(self, sql: str, args: Iterable[Any] = ()) -> sqlite3.Cursor:
        with self._lock:
            return self._conn.execute(sql, tuple(args))

    def insert(self, table: str, row: Dict[str, Any]) -> int:
        cols = ",".join(row)
        qs = ",".join("?" for _ in row)
        cur = self.execute(f"INSERT INTO {table} ({cols}) VALUES ({qs})", [_enc(v) for v in row.values()])
        return int(cur.lastrowid)

    def upsert(self, table: str, row: Dict[str, Any]) -> None:
        cols = ",".join(row)
        qs = ",".join("?" for _ in row)
        self.execute(f"INSERT OR REPLACE INTO {table} ({cols}) VALUES ({qs})", [_enc(v) for v in row.values()])

    def update(self, table: str, key: str, key_val: Any, fields: Dict[str, Any]) -> None:
        if not fields:
            return
        sets = ",".join(f"{k}=?" for k in fields)
        self.execute(f"UPDATE {table} SET {sets} WHERE {key}=?", [_enc(v) for v in fields.values()] + [key_val])

    def one(self, sql: str, args: Iterable[Any] = ()) -> Optional[Dict[str, Any]]:
        r = self.execute(sql, args).fetchone()
        return dict(r) if r is not None else None

    def all(self, sql: str, args: Iterable[Any] = ()) -> List[Dict[str, Any]]:
        return [dict(r) for r in self.execute(sql, args).fetchall()]

    def kv_get(self, key: str, default: Any = None) -> Any:
        r = self.one("SELECT value FROM kv WHERE key=?", [key])
        return json.loads(r["value"]) if r else default

    def kv_set(self, key: str, value: Any) -> None:
        self.upsert("kv", {"key": key, "value": json.dumps(value)})

    def close(self) -> None:
        with self._lock:
            self._conn.close()


def _enc(v: Any) -> Any:
    if isinstance(v, (dict, list)):
        return json.dumps(v, default=str)
    if isinstance(v, bool):
        return int(v)
    return v


def dec(v: Any, default: Any = None) -> Any:
    if v is None:
        return default
    if isinstance(v, (bytes, bytearray)):
        return v
    try:
        return json.loads(v)
    except (TypeError, ValueError):
        return v


def now() -> float:
    return time.time()
