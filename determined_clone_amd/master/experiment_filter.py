"""Experiment filter DSL of the experiment list / search (reference
``master/internal/experiment_filter.go:55-478``, used by ``SearchExperiments`` in
``api_experiment.go:2557-2565``), compiled to one sqlite WHERE clause with bound parameters.

The JSON the web UI and SDK send::

    {"filterGroup": {"kind": "group", "conjunction": "and" | "or", "children": [
        {"kind": "field", "location": "LOCATION_TYPE_EXPERIMENT", "columnName": "name",
         "type": "COLUMN_TYPE_TEXT", "operator": "contains", "value": "resnet"},
        {"kind": "group", ...}]},
     "showArchived": false}

* experiment columns (``id``, ``name``, ``description``, ``tags``, ``state``, ``startTime``, ``duration``,
  ``numTrials``, ``progress``, ``user``, ``forkedFrom``, ``resourcePool``, ``projectId``,
  ``checkpointSize``, ``checkpointCount``, ``searcherType``, ``searcherMetric``,
  ``searcherMetricsVal``, ``externalExperimentId``, ``externalTrialId``) -- the same names as
  ``expColumnNameToSQL``; anything else is an error (no user text ever becomes SQL);
* ``hp.<path>`` (``LOCATION_TYPE_HYPERPARAMETERS``): typed comparison against the experiment
  config's hyperparameter definition -- ``const`` values, ``categorical`` value lists and
  ``int`` / ``double`` / ``log`` ranges;
* ``<group>.<metric>.<min|max|mean|last>`` (``LOCATION_TYPE_VALIDATIONS`` / ``_TRAINING`` /
  ``_CUSTOM_METRIC``): the best trial's summary metrics (``training`` -> the training group,
  ``validation`` -> the validation group, any other name a custom group);
* operators ``=``, ``!=``, ``<``, ``<=``, ``>``, ``>=``, ``contains``, ``notContains``, ``isEmpty``,
  ``notEmpty``; nested groups with ``and`` / ``or``.

The clause runs over ``experiments e LEFT JOIN trials bt`` where ``bt`` is the experiment's best
trial (:data:`FROM_BEST_TRIAL`). Differences from the reference, on purpose: a numeric
``contains`` on a categorical hyperparameter matches numeric members (Postgres' ``jsonb ? '8'``
only matches string members, so it never did), and ``contains`` / ``notContains`` on a range
hyperparameter test ``minval <= v <= maxval`` (the reference's ``minval <= v OR maxval >= v``
holds for nearly every value).
"""
import datetime
import json
import re
from typing import Any, Dict, List, Optional, Tuple, Union

OPS = {"=": "=", "!=": "!=", "<": "<", "<=": "<=", ">": ">", ">=": ">="}
EMPTY_OPS = ("isEmpty", "notEmpty")
ALL_OPS = set(OPS) | {"contains", "notContains"} | set(EMPTY_OPS)

# the best trial of an experiment: lowest searcher metric (or highest when smaller_is_better is
# false) -- the reference keeps it as experiments.best_trial_id
_BEST_TRIAL = (
    "(CASE WHEN COALESCE(json_extract(e.config, '$.searcher.smaller_is_better'), 1) "
    "THEN (SELECT t.id FROM trials t WHERE t.experiment_id = e.id AND t.best_validation IS NOT NULL "
    "ORDER BY t.best_validation ASC, t.id ASC LIMIT 1) "
    "ELSE (SELECT t.id FROM trials t WHERE t.experiment_id = e.id AND t.best_validation IS NOT NULL "
    "ORDER BY t.best_validation DESC, t.id ASC LIMIT 1) END)")
FROM_BEST_TRIAL = f"experiments e LEFT JOIN trials bt ON bt.id = {_BEST_TRIAL}"

_NOW = "((julianday('now') - 2440587.5) * 86400.0)"  # epoch seconds, like the stored times

# expColumnNameToSQL: column name -> SQL expression (fixed strings only)
EXPERIMENT_COLUMNS: Dict[str, str] = {
    "id": "e.id",
    "description": "json_extract(e.config, '$.description')",
    "name": "json_extract(e.config, '$.name')",
    "tags": "json_extract(e.config, '$.labels')",
    "searcherType": "json_extract(e.config, '$.searcher.name')",
    "searcherMetric": "json_extract(e.config, '$.searcher.metric')",
    "startTime": "e.start_time",
    "endTime": "e.end_time",
    "duration": f"(COALESCE(e.end_time, {_NOW}) - e.start_time)",
    "state": "e.state",
    "numTrials": "(SELECT COUNT(*) FROM trials t WHERE t.experiment_id = e.id)",
    "progress": "CAST(ROUND(COALESCE(e.progress, 0) * 100) AS INTEGER)",
    "user": "e.owner_id",
    "forkedFrom": "e.parent_id",
    "resourcePool": "json_extract(e.config, '$.resources.resource_pool')",
    "projectId": "e.project_id",
    "checkpointSize": "(SELECT COALESCE(SUM(c.size), 0) FROM checkpoints c WHERE c.experiment_id = e.id "
                      "AND COALESCE(c.state, '') != 'DELETED')",
    "checkpointCount": "(SELECT COUNT(*) FROM checkpoints c WHERE c.experiment_id = e.id "
                       "AND COALESCE(c.state, '') != 'DELETED')",
    "searcherMetricsVal": "bt.best_validation",
    "externalExperimentId": "e.external_experiment_id",
    "externalTrialId": "bt.external_trial_id",
}
_TIME_COLUMNS = ("startTime", "endTime")

# parseMetricsName's pattern (unanchored at the end, like Go's FindStringSubmatch)
_METRIC_ID = re.compile(r"([\x20-\x7e]+?)\.([\x20-\x7e]+)\.(min|max|mean|last)")
# summary_metrics group keys of master/core.py report_metrics
_GROUP_KEYS = {"training": "training_metrics", "avg_metrics": "training_metrics",
               "validation": "validation_metrics"}


class FilterError(ValueError):
    """The filter JSON is malformed (HTTP 400 at the API)."""


def parse_metric_name(name: str) -> Tuple[str, str, str]:
    """``training.loss.min`` -> ``(training_metrics, loss, min)``; ``group_b.value.a.last`` ->
    ``(group_b, value.a, last)`` (reference ``parseMetricsName``)."""
    m = _METRIC_ID.search(name)
    if m is None or m.start() != 0:
        raise FilterError(f"{name} is not a valid metrics id")
    grp, metric, qual = m.group(1), m.group(2), m.group(3)
    return _GROUP_KEYS.get(grp, grp), metric, qual


def _json_path(*keys: str) -> str:
    for k in keys:
        if '"' in k or "\\" in k:
            raise FilterError(f"invalid name {k!r}")
    return "$" + "".join(f'."{k}"' for k in keys)


def _to_epoch(v: Any) -> Any:
    """ISO-8601 timestamps (the UI's date filters) -> epoch seconds (our stored times)."""
    if isinstance(v, str):
        try:
            s = v.replace("Z", "+00:00")
            m = re.match(r"(.*\.\d{6})\d+(.*)", s)  # Go's nanoseconds -> microseconds
            if m:
                s = m.group(1) + m.group(2)
            d = datetime.datetime.fromisoformat(s)
            if d.tzinfo is None:
                d = d.replace(tzinfo=datetime.timezone.utc)
            return d.timestamp()
        except ValueError:
            return v
    return v


class _Compiler:
    def __init__(self) -> None:
        self.params: List[Any] = []

    def p(self, v: Any) -> str:
        if isinstance(v, bool):
            v = int(v)
        elif isinstance(v, (dict, list)):
            v = json.dumps(v)
        self.params.append(v)
        return "?"

    # --------------------------------------------------------------------- nodes
    def node(self, n: Dict[str, Any]) -> str:
        if not isinstance(n, dict):
            raise FilterError("filter nodes must be objects")
        kind = n.get("kind")
        if kind == "group":
            return self.group(n)
        if kind == "field":
            return self.field(n)
        raise FilterError(f"invalid filter kind {kind!r}")

    def group(self, n: Dict[str, Any]) -> str:
        conj = n.get("conjunction")
        if conj is None:
            raise FilterError("group specified with no conjunction")
        if conj not in ("and", "or"):
            raise FilterError(f"invalid conjunction value {conj}")
        children = n.get("children") or []
        if not children:
            return "(1)"
        sep = " AND " if conj == "and" else " OR "
        return "(" + sep.join(f"({self.node(c)})" for c in children) + ")"

    def field(self, n: Dict[str, Any]) -> str:
        op = n.get("operator")
        if op is None:
            raise FilterError("field specified with value but no operator")
        value = n.get("value")
        if value is None and op not in EMPTY_OPS:
            return "(1)"  # an unfinished filter row in the UI matches everything
        if op not in ALL_OPS:
            raise FilterError(f"invalid operator {op}")
        loc = n.get("location") or "LOCATION_TYPE_EXPERIMENT"
        col = str(n.get("columnName") or "")
        ctype = n.get("type") or "COLUMN_TYPE_UNSPECIFIED"
        if loc == "LOCATION_TYPE_EXPERIMENT":
            return self.experiment_field(col, op, value)
        if loc in ("LOCATION_TYPE_VALIDATIONS", "LOCATION_TYPE_TRAINING", "LOCATION_TYPE_CUSTOM_METRIC"):
            return self.metric_field(col, op, value, ctype)
        if loc == "LOCATION_TYPE_HYPERPARAMETERS":
            return self.hp_field(col, op, value, ctype)
        raise FilterError(f"invalid location {loc!r}")

    def experiment_field(self, col: str, op: str, value: Any) -> str:
        sql = EXPERIMENT_COLUMNS.get(col)
        if sql is None:
            raise FilterError(f"invalid experiment column {col}")
        if op == "contains":
            return f"{sql} LIKE {self.p(f'%{value}%')}"
        if op == "notContains":
            return f"{sql} NOT LIKE {self.p(f'%{value}%')}"
        if op == "isEmpty":
            return f"({sql} IS NULL OR {sql} = '' OR {sql} = '[]')"
        if op == "notEmpty":
            return f"({sql} IS NOT NULL AND {sql} != '' AND {sql} != '[]')"
        if col in _TIME_COLUMNS:
            value = _to_epoch(value)
        return f"{sql} {OPS[op]} {self.p(value)}"

    def metric_field(self, col: str, op: str, value: Any, ctype: str) -> str:
        grp, name, qual = parse_metric_name(col)
        base = _json_path(grp, name)
        if qual == "mean":  # stored as sum / count (master/core.py); a stored mean wins
            expr = (f"COALESCE(json_extract(bt.summary_metrics, {self.p(base + '.mean')}), "
                    f"json_extract(bt.summary_metrics, {self.p(base + '.sum')}) * 1.0 / "
                    f"NULLIF(json_extract(bt.summary_metrics, {self.p(base + '.count')}), 0))")
        else:
            expr = f"json_extract(bt.summary_metrics, {self.p(base + '.' + qual)})"
        if ctype == "COLUMN_TYPE_NUMBER":
            expr = f"CAST({expr} AS REAL)"
        if op == "contains":
            return f"{expr} LIKE {self.p(f'%{value}%')}"
        if op == "notContains":
            return f"{expr} NOT LIKE {self.p(f'%{value}%')}"
        if op == "isEmpty":
            return f"{expr} IS NULL"
        if op == "notEmpty":
            return f"{expr} IS NOT NULL"
        return f"{expr} {OPS[op]} {self.p(value)}"

    def hp_field(self, col: str, op: str, value: Any, ctype: str) -> str:
        keys = col[3:].split(".") if col.startswith("hp.") else col.split(".")
        if not all(keys):
            raise FilterError(f"invalid hyperparameter {col!r}")
        base = "$.hyperparameters" + _json_path(*keys)[1:]

        def h(sub: str = "") -> str:
            return f"json_extract(e.config, {self.p(base + ('.' + sub if sub else ''))})"

        def member(v: Any) -> str:  # v is an element of the categorical vals list
            return (f"EXISTS (SELECT 1 FROM json_each(e.config, {self.p(base + '.vals')}) j "
                    f"WHERE j.value = {self.p(v)} OR CAST(j.value AS TEXT) = {self.p(str(v))})")

        kind = lambda t: f"{h('type')} = {self.p(t)}"  # noqa: E731
        rng = lambda: f"{h('type')} IN ('int', 'double', 'log')"  # noqa: E731 (params in order)
        if ctype in ("COLUMN_TYPE_TEXT", "COLUMN_TYPE_DATE"):
            if op in EMPTY_OPS:
                isn = "IS NULL" if op == "isEmpty" else "IS NOT NULL"
                return (f"(CASE WHEN {kind('const')} THEN {h('val')} {isn} "
                        f"WHEN {kind('categorical')} THEN {h('vals')} {isn} ELSE 0 END)")
            if op == "contains":
                return (f"(CASE WHEN {kind('const')} THEN {h('val')} LIKE {self.p(f'%{value}%')} "
                        f"WHEN {kind('categorical')} THEN {member(value)} ELSE 0 END)")
            if op == "notContains":
                return (f"(CASE WHEN {kind('const')} THEN {h('val')} NOT LIKE {self.p(f'%{value}%')} "
                        f"WHEN {kind('categorical')} THEN NOT {member(value)} ELSE 0 END)")
            return f"(CASE WHEN {kind('const')} THEN {h('val')} {OPS[op]} {self.p(value)} ELSE 0 END)"
        # numeric (the default column type)
        if op in EMPTY_OPS:
            isn = "IS NULL" if op == "isEmpty" else "IS NOT NULL"
            return (f"(CASE WHEN {kind('const')} THEN CAST({h('val')} AS REAL) {isn} "
                    f"WHEN {kind('categorical')} THEN {h('vals')} {isn} "
                    f"WHEN {rng()} THEN {h()} {isn} ELSE 0 END)")
        if op == "contains":
            return (f"(CASE WHEN {kind('categorical')} THEN {member(value)} "
                    f"WHEN {rng()} THEN (CAST({h('minval')} AS REAL) <= {self.p(value)} AND "
                    f"CAST({h('maxval')} AS REAL) >= {self.p(value)}) ELSE 0 END)")
        if op == "notContains":
            return (f"(CASE WHEN {kind('categorical')} THEN NOT {member(value)} "
                    f"WHEN {rng()} THEN (CAST({h('minval')} AS REAL) > {self.p(value)} OR "
                    f"CAST({h('maxval')} AS REAL) < {self.p(value)}) ELSE 0 END)")
        o = OPS[op]
        return (f"(CASE WHEN {kind('const')} THEN CAST({h('val')} AS REAL) {o} {self.p(value)} "
                f"WHEN {rng()} THEN (CAST({h('minval')} AS REAL) {o} {self.p(value)} OR "
                f"CAST({h('maxval')} AS REAL) {o} {self.p(value)}) ELSE 0 END)")


def compile_filter(root: Union[str, Dict[str, Any]]) -> Tuple[str, List[Any]]:
    """``(where_sql, params)`` of an ``experimentFilterRoot`` (JSON text or dict) over
    :data:`FROM_BEST_TRIAL`; archived experiments are excluded unless ``showArchived``."""
    if isinstance(root, str):
        try:
            root = json.loads(root)
        except json.JSONDecodeError as e:
            raise FilterError(f"filter is not JSON: {e}") from e
    if not isinstance(root, dict):
        raise FilterError("filter must be a JSON object")
    c = _Compiler()
    fg = root.get("filterGroup")
    where = c.node(fg) if fg is not None else "(1)"
    if not root.get("showArchived"):
        where = f"({where}) AND (e.archived = 0)"
    return where, c.params


def bulk_filter_sql(f: Optional[Dict[str, Any]]) -> Tuple[str, List[Any]]:
    """WHERE clause of ``BulkExperimentFilters`` (the bulk actions' and LaunchTensorboard's
    ``filters``; reference ``experiment/bulk_action.go:75-115``): description / name substrings
    (case-insensitive), every label present, archived, states, owners, project, excluded ids."""
    f = f or {}
    conds, params = ["1"], []
    if f.get("excluded_experiment_ids"):
        ids = [int(i) for i in f["excluded_experiment_ids"]]
        conds.append(f"e.id NOT IN ({','.join('?' * len(ids))})")
        params += ids
    if f.get("description"):
        conds.append("json_extract(e.config, '$.description') LIKE ('%' || ? || '%')")
        params.append(f["description"])
    if f.get("name"):
        conds.append("json_extract(e.config, '$.name') LIKE ('%' || ? || '%')")
        params.append(f["name"])
    for label in f.get("labels") or []:
        conds.append("EXISTS (SELECT 1 FROM json_each(e.config, '$.labels') j WHERE j.value = ?)")
        params.append(label)
    if f.get("archived") is not None:
        conds.append("e.archived = ?")
        params.append(1 if f["archived"] else 0)
    if f.get("states"):
        st = [str(s)[len("STATE_"):] if str(s).startswith("STATE_") else str(s) for s in f["states"]]
        conds.append(f"e.state IN ({','.join('?' * len(st))})")
        params += st
    if f.get("user_ids"):
        ids = [int(i) for i in f["user_ids"]]
        conds.append(f"e.owner_id IN ({','.join('?' * len(ids))})")
        params += ids
    if f.get("project_id"):
        conds.append("e.project_id = ?")
        params.append(int(f["project_id"]))
    return " AND ".join(conds), params
