"""REST routes for user groups, roles and role assignments (reference: ``master/internal/usergroup/
api_groups.go``, ``master/internal/rbac/api_rbac.go``; paths from ``api.proto``: ``/api/v1/groups``,
``/api/v1/roles/...``, ``/api/v1/permissions/summary``). Imported by ``server`` to register them."""
from typing import Any, Dict, List, Optional

from determined_clone_amd.master import rbac
from determined_clone_amd.master.server import HTTPError, Req, _int, _paginate, require, route


def _group_api(r: Req, g: Dict[str, Any], with_users: bool = False) -> Dict[str, Any]:
    members = r.m.db.all("SELECT u.* FROM users u JOIN group_members gm ON gm.user_id=u.id "
                         "WHERE gm.group_id=? ORDER BY u.id", [g["id"]])
    out: Dict[str, Any] = {"groupId": g["id"], "name": g["name"], "numMembers": len(members)}
    if with_users:
        out["users"] = [{"id": u["id"], "username": u["username"]} for u in members]
    return out


def _group(r: Req, gid: Any) -> Dict[str, Any]:
    g = r.m.db.one("SELECT * FROM groups WHERE id=?", [_int(gid)])
    if g is None:
        raise HTTPError(404, f"group {gid} not found")
    return g


def _user_ids(r: Req, ids: Optional[List[Any]]) -> List[int]:
    out = []
    for uid in ids or []:
        if r.m.db.one("SELECT id FROM users WHERE id=?", [_int(uid)]) is None:
            raise HTTPError(404, f"user {uid} not found")
        out.append(_int(uid))
    return out


# ---------------------------------------------------------------------------- groups
@route("POST", "/api/v1/groups")
def create_group(r: Req) -> Any:
    require(r, "UPDATE_GROUP")
    name = r.body.get("name")
    if not name:
        raise HTTPError(400, "group name required")
    if r.m.db.one("SELECT id FROM groups WHERE name=?", [name]):
        raise HTTPError(409, f"group {name} already exists")
    gid = r.m.db.insert("groups", {"name": name})
    for uid in _user_ids(r, r.body.get("addUsers")):
        r.m.db.upsert("group_members", {"group_id": gid, "user_id": uid})
    g = _group(r, gid)
    return {"group": _group_api(r, g, True)}


@route("POST", "/api/v1/groups/search")
def search_groups(r: Req) -> Any:
    rows = r.m.db.all("SELECT * FROM groups ORDER BY id")
    uid = r.body.get("userId")
    if uid is not None:
        mine = {x["group_id"] for x in r.m.db.all("SELECT group_id FROM group_members WHERE user_id=?", [_int(uid)])}
        rows = [g for g in rows if g["id"] in mine]
    if r.body.get("name"):
        rows = [g for g in rows if g["name"] == r.body["name"]]
    r.q.setdefault("offset", [str(r.body.get("offset", 0))])
    r.q.setdefault("limit", [str(r.body.get("limit", 0))])
    p = _paginate([{"group": _group_api(r, g)} for g in rows], r)
    return {"groups": p["items"], "pagination": p["pagination"]}


@route("GET", "/api/v1/groups/{gid}")
def get_group(r: Req) -> Any:
    return {"group": _group_api(r, _group(r, r.p["gid"]), True)}


@route("PUT", "/api/v1/groups/{gid}")
def update_group(r: Req) -> Any:
    require(r, "UPDATE_GROUP")
    g = _group(r, r.p["gid"])
    if r.body.get("name"):
        other = r.m.db.one("SELECT id FROM groups WHERE name=?", [r.body["name"]])
        if other and other["id"] != g["id"]:
            raise HTTPError(409, f"group {r.body['name']} already exists")
        r.m.db.update("groups", "id", g["id"], {"name": r.body["name"]})
    for uid in _user_ids(r, r.body.get("addUsers")):
        r.m.db.upsert("group_members", {"group_id": g["id"], "user_id": uid})
    for uid in _user_ids(r, r.body.get("removeUsers")):
        r.m.db.execute("DELETE FROM group_members WHERE group_id=? AND user_id=?", [g["id"], uid])
    return {"group": _group_api(r, _group(r, g["id"]), True)}


@route("DELETE", "/api/v1/groups/{gid}")
def delete_group(r: Req) -> Any:
    require(r, "UPDATE_GROUP")
    g = _group(r, r.p["gid"])
    r.m.db.execute("DELETE FROM group_members WHERE group_id=?", [g["id"]])
    r.m.db.execute("DELETE FROM role_assignments WHERE group_id=?", [g["id"]])
    r.m.db.execute("DELETE FROM groups WHERE id=?", [g["id"]])
    return {}


# ---------------------------------------------------------------------------- roles
@route("POST", "/api/v1/roles/search")
def list_roles(r: Req) -> Any:
    return {"roles": [x.api() for x in rbac.ROLES.values()]}


@route("POST", "/api/v1/roles/search/by-ids")
def roles_by_id(r: Req) -> Any:
    out = []
    for rid in r.body.get("roleIds", []):
        role = rbac.ROLES.get(_int(rid))
        if role is None:
            raise HTTPError(404, f"role {rid} not found")
        d = role.api()
        d["assignments"] = [{"userId": a["user_id"], "groupId": a["group_id"], "scopeWorkspaceId": a["workspace_id"]}
                            for a in r.m.db.all("SELECT * FROM role_assignments WHERE role=?", [str(role.id)])]
        out.append(d)
    return {"roles": out}


@route("POST", "/api/v1/roles/search/by-assignability")
def roles_assignable(r: Req) -> Any:
    ws = r.body.get("workspaceId")
    roles = [x for x in rbac.ROLES.values() if (x.workspace_assignable if ws else x.global_assignable)]
    return {"roles": [x.api() for x in roles]}


def _assignment_api(a: Dict[str, Any]) -> Dict[str, Any]:
    role = rbac.ROLES.get(int(a["role"]) if "role" in a else a["role_id"])
    return {"role": role.api() if role else None, "scopeWorkspaceId": a["workspace_id"],
            "scopeCluster": a["workspace_id"] is None, "groupId": a.get("group_id"),
            "userId": a.get("user_id")}


@route("GET", "/api/v1/roles/search/by-user/{uid}")
def roles_of_user(r: Req) -> Any:
    uid = _int(r.p["uid"])
    if r.m.db.one("SELECT id FROM users WHERE id=?", [uid]) is None:
        raise HTTPError(404, f"user {uid} not found")
    return {"roles": [_assignment_api(a) for a in r.m.authz.assignments_for_user(uid)]}


@route("GET", "/api/v1/roles/search/by-group/{gid}")
def roles_of_group(r: Req) -> Any:
    g = _group(r, r.p["gid"])
    return {"roles": [_assignment_api(a) for a in
                      r.m.db.all("SELECT * FROM role_assignments WHERE group_id=?", [g["id"]])]}


@route("GET", "/api/v1/roles/workspace/{wid}")
def roles_in_workspace(r: Req) -> Any:
    wid = _int(r.p["wid"])
    rows = r.m.db.all("SELECT * FROM role_assignments WHERE workspace_id=?", [wid])
    users = sorted({a["user_id"] for a in rows if a["user_id"] is not None})
    groups = sorted({a["group_id"] for a in rows if a["group_id"] is not None})
    return {"usersAssignedDirectly": [{"id": u} for u in users],
            "groups": [{"groupId": g} for g in groups],
            "assignments": [_assignment_api(a) for a in rows]}


def _apply_assignments(r: Req, add: bool) -> None:
    for key, who in (("userRoleAssignments", "userId"), ("groupRoleAssignments", "groupId")):
        for item in r.body.get(key, []) or []:
            ra = item.get("roleAssignment", {})
            role_id = _int((ra.get("role") or {}).get("roleId"))
            ws = ra.get("scopeWorkspaceId")
            ws = _int(ws) if ws is not None else None
            # assigning inside a workspace needs ASSIGN_ROLES there; cluster-wide needs UPDATE_ROLES
            if ws is None:
                require(r, "UPDATE_ROLES")
            else:
                require(r, "ASSIGN_ROLES", ws)
            uid = _int(item[who]) if who == "userId" else None
            gid = _int(item[who]) if who == "groupId" else None
            if gid is not None:
                _group(r, gid)
            try:
                if add:
                    r.m.authz.assign(role_id, user_id=uid, group_id=gid, workspace_id=ws)
                else:
                    r.m.authz.unassign(role_id, user_id=uid, group_id=gid, workspace_id=ws)
            except ValueError as e:
                raise HTTPError(400, str(e))


@route("POST", "/api/v1/roles/add-assignments")
def add_assignments(r: Req) -> Any:
    _apply_assignments(r, True)
    return {}


@route("POST", "/api/v1/roles/remove-assignments")
def remove_assignments(r: Req) -> Any:
    _apply_assignments(r, False)
    return {}


@route("GET", "/api/v1/permissions/summary")
def permissions_summary(r: Req) -> Any:
    return r.m.authz.summary(r.user)
