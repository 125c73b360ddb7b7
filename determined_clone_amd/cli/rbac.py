"""``det user-group`` and ``det rbac`` (reference: ``harness/determined/cli/user_groups.py``,
``harness/determined/cli/rbac.py``) over the master's groups / roles routes."""
import argparse
from typing import Any, Dict, List, Optional

from determined_clone_amd.cli.cli import render_table, session


def _user_id(s: Any, username: str) -> int:
    for u in s.get("/api/v1/users")["users"]:
        if u["username"] == username:
            return u["id"]
    raise SystemExit(f"user {username} not found")


def _group_id(s: Any, name: str) -> int:
    gs = s.post("/api/v1/groups/search", {"name": name})["groups"]
    if not gs:
        raise SystemExit(f"group {name} not found")
    return gs[0]["group"]["groupId"]


def _workspace_id(s: Any, name: Optional[str]) -> Optional[int]:
    if not name:
        return None
    for w in s.get("/api/v1/workspaces")["workspaces"]:
        if w["name"] == name:
            return w["id"]
    raise SystemExit(f"workspace {name} not found")


def _role(s: Any, name: str) -> Dict[str, Any]:
    for r in s.post("/api/v1/roles/search", {})["roles"]:
        if r["name"].lower() == name.lower():
            return r
    raise SystemExit(f"role {name} not found")


# ---------------------------------------------------------------------------- user groups
def group_create(args: argparse.Namespace) -> None:
    s = session(args)
    ids = [_user_id(s, u) for u in args.add_user or []]
    g = s.post("/api/v1/groups", {"name": args.group_name, "addUsers": ids})["group"]
    print(f"user group with name {g['name']} and ID {g['groupId']} created")


def group_list(args: argparse.Namespace) -> None:
    s = session(args)
    body: Dict[str, Any] = {}
    if args.groups_user_belongs_to:
        body["userId"] = _user_id(s, args.groups_user_belongs_to)
    rows = [g["group"] for g in s.post("/api/v1/groups/search", body)["groups"]]
    render_table(rows, ["groupId", "name", "numMembers"], args.json)


def group_describe(args: argparse.Namespace) -> None:
    s = session(args)
    g = s.get(f"/api/v1/groups/{_group_id(s, args.group_name)}")["group"]
    if args.json:
        render_table([g], [], True)
        return
    print(f"group ID: {g['groupId']}   group name: {g['name']}")
    render_table(g.get("users", []), ["id", "username"])


def _group_users(add: bool):
    def f(args: argparse.Namespace) -> None:
        s = session(args)
        gid = _group_id(s, args.group_name)
        ids = [_user_id(s, u) for u in args.usernames.split(",")]
        s.put(f"/api/v1/groups/{gid}", {"addUsers" if add else "removeUsers": ids})
        print(f"user group {args.group_name}: {'added' if add else 'removed'} {args.usernames}")
    return f


def group_change_name(args: argparse.Namespace) -> None:
    s = session(args)
    s.put(f"/api/v1/groups/{_group_id(s, args.old_group_name)}", {"name": args.new_group_name})
    print(f"user group {args.old_group_name} renamed to {args.new_group_name}")


def group_delete(args: argparse.Namespace) -> None:
    s = session(args)
    s.delete(f"/api/v1/groups/{_group_id(s, args.group_name)}")
    print(f"user group {args.group_name} deleted")


# ---------------------------------------------------------------------------- rbac
def my_permissions(args: argparse.Namespace) -> None:
    s = session(args)
    summ = s.get("/api/v1/permissions/summary")
    names = {r["roleId"]: r for r in summ["roles"]}
    rows: List[Dict[str, Any]] = []
    for a in summ["assignments"]:
        role = names[a["roleId"]]
        scope = "cluster" if a["scopeCluster"] else ",".join(str(w) for w in a["scopeWorkspaceIds"])
        for p in role["permissions"]:
            rows.append({"role": role["name"], "scope": scope, "permission": p["name"]})
    render_table(rows, ["role", "scope", "permission"], args.json)


def list_roles(args: argparse.Namespace) -> None:
    s = session(args)
    rows = [{"roleId": r["roleId"], "name": r["name"], "permissions": len(r["permissions"]),
             "cluster": r["scopeTypeMask"]["cluster"], "workspace": r["scopeTypeMask"]["workspace"]}
            for r in s.post("/api/v1/roles/search", {})["roles"]]
    render_table(rows, ["roleId", "name", "permissions", "cluster", "workspace"], args.json)


def describe_role(args: argparse.Namespace) -> None:
    s = session(args)
    r = s.post("/api/v1/roles/search/by-ids", {"roleIds": [_role(s, args.role_name)["roleId"]]})["roles"][0]
    if args.json:
        render_table([r], [], True)
        return
    print(f"role {r['name']} (id {r['roleId']})")
    render_table([{"id": p["id"], "name": p["name"]} for p in r["permissions"]], ["id", "name"])
    render_table(r["assignments"], ["userId", "groupId", "scopeWorkspaceId"])


def _assignment_rows(items: List[Dict[str, Any]]) -> List[Dict[str, Any]]:
    return [{"role": (a["role"] or {}).get("name"), "workspace": a["scopeWorkspaceId"],
             "cluster": a["scopeCluster"], "via_group": a.get("groupId")} for a in items]


def list_users_roles(args: argparse.Namespace) -> None:
    s = session(args)
    roles = s.get(f"/api/v1/roles/search/by-user/{_user_id(s, args.username)}")["roles"]
    render_table(_assignment_rows(roles), ["role", "workspace", "cluster", "via_group"], args.json)


def list_groups_roles(args: argparse.Namespace) -> None:
    s = session(args)
    roles = s.get(f"/api/v1/roles/search/by-group/{_group_id(s, args.group_name)}")["roles"]
    render_table(_assignment_rows(roles), ["role", "workspace", "cluster"], args.json)


def _assign(add: bool):
    def f(args: argparse.Namespace) -> None:
        s = session(args)
        if bool(args.username_to_assign) == bool(args.group_name_to_assign):
            raise SystemExit("give exactly one of --username-to-assign / --group-name-to-assign")
        ra = {"role": {"roleId": _role(s, args.role_name)["roleId"]},
              "scopeWorkspaceId": _workspace_id(s, args.workspace_name)}
        if args.username_to_assign:
            body = {"userRoleAssignments": [{"userId": _user_id(s, args.username_to_assign), "roleAssignment": ra}]}
        else:
            body = {"groupRoleAssignments": [{"groupId": _group_id(s, args.group_name_to_assign), "roleAssignment": ra}]}
        s.post("/api/v1/roles/add-assignments" if add else "/api/v1/roles/remove-assignments", body)
        who = args.username_to_assign or args.group_name_to_assign
        where = f"workspace {args.workspace_name}" if args.workspace_name else "cluster"
        print(f"{'assigned' if add else 'removed'} role {args.role_name} {'to' if add else 'from'} {who} ({where})")
    return f


def register(cmd: Any, group: Any) -> None:
    """Add the ``user-group`` and ``rbac`` command groups to the ``det`` parser."""
    g = group("user-group")
    sp = cmd(g, "create", group_create); sp.add_argument("group_name"); sp.add_argument("--add-user", action="append")
    sp = cmd(g, "list ls", group_list); sp.add_argument("--groups-user-belongs-to")
    sp = cmd(g, "describe", group_describe); sp.add_argument("group_name")
    sp = cmd(g, "add-user", _group_users(True)); sp.add_argument("group_name"); sp.add_argument("usernames", help="comma-separated")
    sp = cmd(g, "remove-user", _group_users(False)); sp.add_argument("group_name"); sp.add_argument("usernames", help="comma-separated")
    sp = cmd(g, "change-name", group_change_name); sp.add_argument("old_group_name"); sp.add_argument("new_group_name")
    sp = cmd(g, "delete", group_delete); sp.add_argument("group_name")

    r = group("rbac")
    cmd(r, "my-permissions", my_permissions)
    cmd(r, "list-roles", list_roles)
    sp = cmd(r, "describe-role", describe_role); sp.add_argument("role_name")
    sp = cmd(r, "list-users-roles", list_users_roles); sp.add_argument("username")
    sp = cmd(r, "list-groups-roles", list_groups_roles); sp.add_argument("group_name")
    for name, add in (("assign-role", True), ("unassign-role", False)):
        sp = cmd(r, name, _assign(add))
        sp.add_argument("role_name")
        sp.add_argument("--username-to-assign", "-u")
        sp.add_argument("--group-name-to-assign", "-g")
        sp.add_argument("--workspace-name", "-w")
