"""Authorization: user groups, roles, role assignments and permission checks.

Reference: ``master/internal/rbac`` + ``master/internal/usergroup`` (RBAC API,
``proto/src/determined/api/v1/api.proto`` GetGroups/CreateGroup/UpdateGroup/AssignRoles/...,
permission ids in ``proto/src/determined/rbac/v1/rbac.proto``) and the ``security.authz.type``
master setting (``master/internal/config/authz_config.go``: ``basic`` or ``rbac``).

* ``basic`` mode: every active user may do everything except cluster administration
  (users, agents, roles, webhooks, master config), which needs an admin user.
* ``rbac`` mode: a user holds the union of the permissions of the roles assigned to them or to
  any of their groups, either globally or in the workspace of the object acted on. Admin users
  keep every permission (the bootstrap admin must be able to assign the first roles).
"""
from typing import Any, Dict, FrozenSet, Iterable, List, Optional, Tuple

PERMISSIONS: Dict[str, int] = {
    "ADMINISTRATE_USER": 91001,
    "ADMINISTRATE_OAUTH": 91002,
    "CREATE_EXPERIMENT": 2001,
    "VIEW_EXPERIMENT_ARTIFACTS": 2002,
    "VIEW_EXPERIMENT_METADATA": 2003,
    "UPDATE_EXPERIMENT": 2004,
    "UPDATE_EXPERIMENT_METADATA": 2005,
    "DELETE_EXPERIMENT": 2006,
    "CREATE_NSC": 3001,
    "VIEW_NSC": 3002,
    "UPDATE_NSC": 3003,
    "UPDATE_GROUP": 93001,
    "CREATE_WORKSPACE": 94001,
    "VIEW_WORKSPACE": 4002,
    "UPDATE_WORKSPACE": 4003,
    "DELETE_WORKSPACE": 4004,
    "SET_WORKSPACE_AGENT_USER_GROUP": 4005,
    "SET_WORKSPACE_CHECKPOINT_STORAGE_CONFIG": 4006,
    "SET_WORKSPACE_DEFAULT_RESOURCE_POOL": 4007,
    "CREATE_PROJECT": 5001,
    "VIEW_PROJECT": 5002,
    "UPDATE_PROJECT": 5003,
    "DELETE_PROJECT": 5004,
    "ASSIGN_ROLES": 6002,
    "VIEW_MODEL_REGISTRY": 7001,
    "EDIT_MODEL_REGISTRY": 7002,
    "CREATE_MODEL_REGISTRY": 7003,
    "DELETE_MODEL_REGISTRY": 7004,
    "DELETE_MODEL_VERSION": 7005,
    "DELETE_OTHER_USER_MODEL_REGISTRY": 7006,
    "DELETE_OTHER_USER_MODEL_VERSION": 7007,
    "VIEW_MASTER_LOGS": 8001,
    "VIEW_CLUSTER_USAGE": 8002,
    "UPDATE_AGENTS": 8003,
    "VIEW_SENSITIVE_AGENT_INFO": 8004,
    "VIEW_MASTER_CONFIG": 8005,
    "UPDATE_MASTER_CONFIG": 8006,
    "CONTROL_STRICT_JOB_QUEUE": 8101,
    "VIEW_TEMPLATES": 9001,
    "UPDATE_TEMPLATES": 9002,
    "CREATE_TEMPLATES": 9003,
    "DELETE_TEMPLATES": 9004,
    "UPDATE_ROLES": 96001,
    "EDIT_WEBHOOKS": 97001,
    "MODIFY_RP_WORKSPACE_BINDINGS": 10001,
}
_ID_TO_NAME = {v: k for k, v in PERMISSIONS.items()}

# permissions that are cluster-wide by nature (not meaningful inside one workspace)
GLOBAL_ONLY = frozenset({
    "ADMINISTRATE_USER", "ADMINISTRATE_OAUTH", "UPDATE_GROUP", "CREATE_WORKSPACE",
    "VIEW_MASTER_LOGS", "VIEW_CLUSTER_USAGE", "UPDATE_AGENTS", "VIEW_SENSITIVE_AGENT_INFO",
    "VIEW_MASTER_CONFIG", "UPDATE_MASTER_CONFIG", "UPDATE_ROLES", "EDIT_WEBHOOKS",
    "MODIFY_RP_WORKSPACE_BINDINGS", "CONTROL_STRICT_JOB_QUEUE",
})

_VIEW = frozenset({"VIEW_EXPERIMENT_ARTIFACTS", "VIEW_EXPERIMENT_METADATA", "VIEW_NSC",
                   "VIEW_WORKSPACE", "VIEW_PROJECT", "VIEW_MODEL_REGISTRY", "VIEW_TEMPLATES"})
_EDIT = _VIEW | frozenset({
    "CREATE_EXPERIMENT", "UPDATE_EXPERIMENT", "UPDATE_EXPERIMENT_METADATA", "DELETE_EXPERIMENT",
    "CREATE_NSC", "UPDATE_NSC", "CREATE_PROJECT", "UPDATE_PROJECT", "DELETE_PROJECT",
    "EDIT_MODEL_REGISTRY", "CREATE_MODEL_REGISTRY", "DELETE_MODEL_REGISTRY",
    "DELETE_MODEL_VERSION"})
_WS_ADMIN = _EDIT | frozenset({
    "UPDATE_WORKSPACE", "DELETE_WORKSPACE", "SET_WORKSPACE_AGENT_USER_GROUP",
    "SET_WORKSPACE_CHECKPOINT_STORAGE_CONFIG", "SET_WORKSPACE_DEFAULT_RESOURCE_POOL",
    "ASSIGN_ROLES", "DELETE_OTHER_USER_MODEL_REGISTRY", "DELETE_OTHER_USER_MODEL_VERSION",
    "UPDATE_TEMPLATES", "CREATE_TEMPLATES", "DELETE_TEMPLATES"})


class Role:
    __slots__ = ("id", "name", "permissions", "global_assignable", "workspace_assignable")

    def __init__(self, rid: int, name: str, permissions: Iterable[str], global_assignable: bool = True,
                 workspace_assignable: bool = True) -> None:
        self.id = rid
        self.name = name
        self.permissions: FrozenSet[str] = frozenset(permissions)
        self.global_assignable = global_assignable
        self.workspace_assignable = workspace_assignable

    def api(self) -> Dict[str, Any]:
        return {"roleId": self.id, "name": self.name,
                "permissions": [{"id": PERMISSIONS[p], "name": p,
                                 "scopeTypeMask": {"cluster": True, "workspace": p not in GLOBAL_ONLY}}
                                for p in sorted(self.permissions)],
                "scopeTypeMask": {"cluster": self.global_assignable,
                                  "workspace": self.workspace_assignable}}


ROLES: Dict[int, Role] = {r.id: r for r in (
    Role(1, "ClusterAdmin", PERMISSIONS.keys(), workspace_assignable=False),
    Role(2, "WorkspaceAdmin", _WS_ADMIN),
    Role(3, "WorkspaceCreator", {"CREATE_WORKSPACE"}, workspace_assignable=False),
    Role(4, "Viewer", _VIEW),
    Role(5, "Editor", _EDIT),
    Role(6, "EditorRestricted", _EDIT - {"CREATE_NSC", "UPDATE_NSC"}),
)}


def role_by_name(name: str) -> Optional[Role]:
    for r in ROLES.values():
        if r.name.lower() == str(name).lower():
            return r
    return None


def permission_name(p: Any) -> str:
    if isinstance(p, int):
        return _ID_TO_NAME[p]
    p = str(p)
    return p[len("PERMISSION_TYPE_"):] if p.startswith("PERMISSION_TYPE_") else p


class Authz:
    """Permission checks over the master DB (``groups``, ``group_members``, ``role_assignments``)."""

    def __init__(self, db: Any, mode: str = "basic") -> None:
        if mode not in ("basic", "rbac"):
            raise ValueError(f"security.authz.type must be basic or rbac, got {mode!r}")
        self.db = db
        self.mode = mode

    # ------------------------------------------------------------------ queries
    def group_ids(self, user_id: int) -> List[int]:
        return [r["group_id"] for r in self.db.all("SELECT group_id FROM group_members WHERE user_id=?", [user_id])]

    def assignments_for_user(self, user_id: int) -> List[Dict[str, Any]]:
        """Direct and group-inherited assignments: dicts with role_id, workspace_id, group_id."""
        rows = self.db.all("SELECT * FROM role_assignments WHERE user_id=?", [user_id])
        gids = self.group_ids(user_id)
        if gids:
            marks = ",".join("?" * len(gids))
            rows += self.db.all(f"SELECT * FROM role_assignments WHERE group_id IN ({marks})", gids)
        return [{"role_id": int(r["role"]), "workspace_id": r["workspace_id"], "group_id": r["group_id"],
                 "user_id": r["user_id"], "id": r["id"]} for r in rows]

    def permissions(self, user: Dict[str, Any], workspace_id: Optional[int] = None) -> FrozenSet[str]:
        if user.get("admin"):
            return frozenset(PERMISSIONS)
        if self.mode == "basic":
            return frozenset(PERMISSIONS) - GLOBAL_ONLY | {"CREATE_WORKSPACE"}
        out = set()
        for a in self.assignments_for_user(user["id"]):
            role = ROLES.get(a["role_id"])
            if role is None:
                continue
            if a["workspace_id"] is None or (workspace_id is not None and a["workspace_id"] == workspace_id):
                out |= role.permissions
        return frozenset(out)

    def permitted(self, user: Optional[Dict[str, Any]], perm: str, workspace_id: Optional[int] = None) -> bool:
        if user is None:
            return False
        return permission_name(perm) in self.permissions(user, workspace_id)

    # ------------------------------------------------------------------ mutations
    def assign(self, role_id: int, user_id: Optional[int] = None, group_id: Optional[int] = None,
               workspace_id: Optional[int] = None) -> int:
        role = ROLES.get(int(role_id))
        if role is None:
            raise KeyError(f"role {role_id}")
        if (user_id is None) == (group_id is None):
            raise ValueError("an assignment names exactly one of a user or a group")
        if workspace_id is None and not role.global_assignable:
            raise ValueError(f"role {role.name} cannot be assigned cluster-wide")
        if workspace_id is not None and not role.workspace_assignable:
            raise ValueError(f"role {role.name} cannot be assigned to a workspace")
        existing = self.db.one(
            "SELECT id FROM role_assignments WHERE role=? AND user_id IS ? AND group_id IS ? AND workspace_id IS ?",
            [str(role.id), user_id, group_id, workspace_id])
        if existing:
            return existing["id"]
        return self.db.insert("role_assignments", {"role": str(role.id), "user_id": user_id,
                                                   "group_id": group_id, "workspace_id": workspace_id})

    def unassign(self, role_id: int, user_id: Optional[int] = None, group_id: Optional[int] = None,
                 workspace_id: Optional[int] = None) -> int:
        cur = self.db.execute(
            "DELETE FROM role_assignments WHERE role=? AND user_id IS ? AND group_id IS ? AND workspace_id IS ?",
            [str(int(role_id)), user_id, group_id, workspace_id])
        return getattr(cur, "rowcount", 0)

    def summary(self, user: Dict[str, Any]) -> Dict[str, Any]:
        """GetPermissionsSummary: the user's roles and where they apply."""
        assigns = self.assignments_for_user(user["id"])
        if user.get("admin"):
            assigns = [{"role_id": 1, "workspace_id": None, "group_id": None, "user_id": user["id"], "id": 0}] + assigns
        role_ids = sorted({a["role_id"] for a in assigns if a["role_id"] in ROLES})
        return {"roles": [ROLES[r].api() for r in role_ids],
                "assignments": [{"roleId": a["role_id"], "scopeWorkspaceIds": [a["workspace_id"]] if a["workspace_id"] is not None else [],
                                 "scopeCluster": a["workspace_id"] is None, "groupId": a["group_id"]}
                                for a in assigns if a["role_id"] in ROLES],
                "mode": self.mode}
