"""RBAC: user groups, role assignments (cluster / workspace scope, direct / via group) and the
permission checks of the master routes, through the REST API and the ``det`` CLI."""
import os
import shutil
import tempfile

import pytest
import yaml

from determined_clone_amd.cli import cli
from determined_clone_amd.common.api import Session
from determined_clone_amd.errors import APIException
from determined_clone_amd.master import Master, MasterServer
from determined_clone_amd.master import rbac

from test_cluster_e2e import BASE


@pytest.fixture(scope="module")
def cluster():
    tmp = tempfile.mkdtemp(prefix="det-rbac-")
    m = Master(os.path.join(tmp, "m.db"), authz="rbac",
               checkpoint_storage={"type": "shared_fs", "host_path": os.path.join(tmp, "ckpt")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    yield m, tmp
    srv.stop()
    shutil.rmtree(tmp, ignore_errors=True)


def _login(m, user, pw=""):
    s = Session(m.master_url)
    s.token = s.post("/api/v1/auth/login", {"username": user, "password": pw})["token"]
    return s


def _exp_cfg(name):
    cfg = yaml.safe_load(BASE)
    cfg["name"] = name
    cfg["searcher"] = {"name": "single", "metric": "val_loss", "max_length": {"batches": 8}}
    return cfg


def test_role_catalogue():
    names = {r.name for r in rbac.ROLES.values()}
    assert {"ClusterAdmin", "WorkspaceAdmin", "WorkspaceCreator", "Viewer", "Editor", "EditorRestricted"} <= names
    assert rbac.permission_name(2001) == "CREATE_EXPERIMENT"
    assert rbac.permission_name("PERMISSION_TYPE_CREATE_NSC") == "CREATE_NSC"
    assert "CREATE_NSC" not in rbac.role_by_name("editorrestricted").permissions


def test_rbac_workspace_scoped_permissions(cluster):
    m, _ = cluster
    admin = _login(m, "admin")
    admin.post("/api/v1/users", {"user": {"username": "alice"}, "password": "pw"})
    admin.post("/api/v1/users", {"user": {"username": "bob"}, "password": "pw"})
    ws = admin.post("/api/v1/workspaces", {"name": "team-a"})["workspace"]
    proj = admin.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "p1"})["project"]
    alice = _login(m, "alice", "pw")
    uid = {u["username"]: u["id"] for u in admin.get("/api/v1/users")["users"]}

    # no roles: cannot create experiments, workspaces or groups
    with pytest.raises(APIException, match="403|permission"):
        alice.post("/api/v1/experiments", {"config": _exp_cfg("a"), "project_id": proj["id"], "activate": False})
    with pytest.raises(APIException, match="403|permission"):
        alice.post("/api/v1/workspaces", {"name": "alice-ws"})
    with pytest.raises(APIException, match="403|permission"):
        alice.post("/api/v1/groups", {"name": "g"})

    # Editor in team-a only
    editor = rbac.role_by_name("Editor").id
    admin.post("/api/v1/roles/add-assignments", {"userRoleAssignments": [
        {"userId": uid["alice"], "roleAssignment": {"role": {"roleId": editor}, "scopeWorkspaceId": ws["id"]}}]})
    e = alice.post("/api/v1/experiments", {"config": _exp_cfg("a"), "project_id": proj["id"], "activate": False})
    eid = e["experiment"]["id"]
    alice.post(f"/api/v1/experiments/{eid}/kill")
    with pytest.raises(APIException, match="403|permission"):  # default workspace: no role there
        alice.post("/api/v1/experiments", {"config": _exp_cfg("b"), "project_id": 1, "activate": False})
    summ = alice.get("/api/v1/permissions/summary")
    assert summ["mode"] == "rbac" and [r["name"] for r in summ["roles"]] == ["Editor"]
    assert summ["assignments"][0]["scopeWorkspaceIds"] == [ws["id"]]

    # Viewer cannot update; role via a group grants cluster-wide WorkspaceCreator
    bob = _login(m, "bob", "pw")
    viewer = rbac.role_by_name("Viewer").id
    admin.post("/api/v1/roles/add-assignments", {"userRoleAssignments": [
        {"userId": uid["bob"], "roleAssignment": {"role": {"roleId": viewer}, "scopeWorkspaceId": ws["id"]}}]})
    with pytest.raises(APIException, match="403|permission"):
        bob.post(f"/api/v1/experiments/{eid}/pause")
    g = admin.post("/api/v1/groups", {"name": "creators", "addUsers": [uid["bob"]]})["group"]
    assert g["numMembers"] == 1 and g["users"][0]["username"] == "bob"
    creator = rbac.role_by_name("WorkspaceCreator").id
    admin.post("/api/v1/roles/add-assignments", {"groupRoleAssignments": [
        {"groupId": g["groupId"], "roleAssignment": {"role": {"roleId": creator}}}]})
    bob.post("/api/v1/workspaces", {"name": "bob-ws"})
    roles = admin.get(f"/api/v1/roles/search/by-user/{uid['bob']}")["roles"]
    assert {r["role"]["name"] for r in roles} == {"Viewer", "WorkspaceCreator"}
    # a cluster-only role cannot be scoped to a workspace
    with pytest.raises(APIException, match="400|cannot"):
        admin.post("/api/v1/roles/add-assignments", {"groupRoleAssignments": [
            {"groupId": g["groupId"], "roleAssignment": {"role": {"roleId": creator}, "scopeWorkspaceId": ws["id"]}}]})
    # removing the user from the group drops the inherited role
    admin.put(f"/api/v1/groups/{g['groupId']}", {"removeUsers": [uid["bob"]]})
    with pytest.raises(APIException, match="403|permission"):
        bob.post("/api/v1/workspaces", {"name": "bob-ws2"})
    # unassign
    admin.post("/api/v1/roles/remove-assignments", {"userRoleAssignments": [
        {"userId": uid["alice"], "roleAssignment": {"role": {"roleId": editor}, "scopeWorkspaceId": ws["id"]}}]})
    with pytest.raises(APIException, match="403|permission"):
        alice.post("/api/v1/experiments", {"config": _exp_cfg("c"), "project_id": proj["id"], "activate": False})


def test_basic_mode_keeps_cluster_admin_checks(tmp_path):
    m = Master(str(tmp_path / "m.db"), checkpoint_storage={"type": "shared_fs", "host_path": str(tmp_path / "c")})
    srv = MasterServer(m, "127.0.0.1", 0).start()
    try:
        admin = _login(m, "admin")
        admin.post("/api/v1/users", {"user": {"username": "carol"}, "password": "x"})
        carol = _login(m, "carol", "x")
        carol.post("/api/v1/experiments", {"config": _exp_cfg("ok"), "activate": False})  # allowed in basic
        carol.post("/api/v1/workspaces", {"name": "carol-ws"})
        with pytest.raises(APIException, match="403|permission"):
            carol.post("/api/v1/groups", {"name": "nope"})
        with pytest.raises(APIException, match="403|permission"):
            carol.post("/api/v1/users", {"user": {"username": "dave"}})
    finally:
        srv.stop()


def test_cli_user_groups_and_rbac(cluster, tmp_path, monkeypatch, capsys):
    m, _ = cluster
    monkeypatch.setattr(cli, "AUTH_FILE", tmp_path / "auth.json")
    base = ["-m", m.master_url, "-u", "admin"]
    admin = _login(m, "admin")
    admin.post("/api/v1/users", {"user": {"username": "erin"}, "password": ""})
    admin.post("/api/v1/workspaces", {"name": "cli-ws"})
    assert cli.main(base + ["user-group", "create", "ml", "--add-user", "erin"]) == 0
    assert cli.main(base + ["user-group", "add-user", "ml", "admin"]) == 0
    assert cli.main(base + ["user-group", "describe", "ml"]) == 0
    out = capsys.readouterr().out
    assert "erin" in out and "admin" in out
    assert cli.main(base + ["rbac", "assign-role", "WorkspaceAdmin", "-g", "ml", "-w", "cli-ws"]) == 0
    assert cli.main(base + ["rbac", "list-users-roles", "erin"]) == 0
    out = capsys.readouterr().out
    assert "WorkspaceAdmin" in out
    assert cli.main(base + ["rbac", "list-roles"]) == 0
    assert cli.main(base + ["rbac", "describe-role", "Viewer"]) == 0
    assert cli.main(["-m", m.master_url, "-u", "erin", "rbac", "my-permissions"]) == 0
    out = capsys.readouterr().out
    assert "CREATE_EXPERIMENT" in out and "ASSIGN_ROLES" in out
    assert cli.main(base + ["rbac", "unassign-role", "WorkspaceAdmin", "-g", "ml", "-w", "cli-ws"]) == 0
    assert cli.main(base + ["user-group", "change-name", "ml", "ml2"]) == 0
    assert cli.main(base + ["user-group", "list"]) == 0
    assert "ml2" in capsys.readouterr().out
    assert cli.main(base + ["user-group", "delete", "ml2"]) == 0


def test_checkpoint_delete_needs_experiment_edit_permission(cluster):
    # reference: master/internal/api_checkpoint.go CheckpointsRemoveFiles -- edit permission on the
    # owning experiment, no model-registry checkpoints, no empty / '..' globs, partial globs update
    # the stored resources
    m, tmp = cluster
    admin = _login(m, "admin")
    admin.post("/api/v1/users", {"user": {"username": "carol"}, "password": "pw"})
    uid = {u["username"]: u["id"] for u in admin.get("/api/v1/users")["users"]}
    ws = admin.post("/api/v1/workspaces", {"name": "team-ck"})["workspace"]
    proj = admin.post(f"/api/v1/workspaces/{ws['id']}/projects", {"name": "pck"})["project"]
    eid = admin.post("/api/v1/experiments", {"config": _exp_cfg("ck"), "project_id": proj["id"],
                                             "activate": False})["experiment"]["id"]
    ckdir = os.path.join(tmp, "ckpt")
    uuids = []
    for i in range(2):
        u = f"00000000-0000-0000-0000-00000000000{i}"
        os.makedirs(os.path.join(ckdir, u, "sub"), exist_ok=True)
        for f in ("state_dict.pth", "sub/extra.bin"):
            with open(os.path.join(ckdir, u, f), "w") as fh:
                fh.write("x" * 10)
        m.db.upsert("checkpoints", {"uuid": u, "experiment_id": eid, "state": "COMPLETED",
                                    "resources": {"state_dict.pth": 10, "sub/extra.bin": 10}, "size": 20})
        uuids.append(u)
    carol = _login(m, "carol", "pw")
    viewer = rbac.role_by_name("Viewer").id
    admin.post("/api/v1/roles/add-assignments", {"userRoleAssignments": [
        {"userId": uid["carol"], "roleAssignment": {"role": {"roleId": viewer}, "scopeWorkspaceId": ws["id"]}}]})
    with pytest.raises(APIException, match="403|permission"):
        carol.post("/api/v1/checkpoints/rm", {"checkpoint_uuids": uuids[:1], "checkpoint_globs": ["**/*"]})
    with pytest.raises(APIException, match="403|permission"):
        carol.patch(f"/api/v1/checkpoints/{uuids[0]}/metadata", {"metadata": {"k": 1}})
    assert os.path.exists(os.path.join(ckdir, uuids[0], "state_dict.pth"))
    for bad in ([""], ["../x"]):
        with pytest.raises(APIException, match="400|glob"):
            admin.post("/api/v1/checkpoints/rm", {"checkpoint_uuids": uuids[:1], "checkpoint_globs": bad})
    # partial delete: only sub/ goes, resources and state follow
    admin.post("/api/v1/checkpoints/rm", {"checkpoint_uuids": uuids[:1], "checkpoint_globs": ["sub"]})
    ck = admin.get(f"/api/v1/checkpoints/{uuids[0]}")["checkpoint"]
    assert ck["state"] == "PARTIALLY_DELETED" and set(ck["resources"]) == {"state_dict.pth"}
    assert not os.path.exists(os.path.join(ckdir, uuids[0], "sub"))
    # a checkpoint registered as a model version cannot be deleted
    admin.post("/api/v1/models", {"name": "ck-model", "workspace_id": ws["id"]})
    admin.post("/api/v1/models/ck-model/versions", {"checkpoint_uuid": uuids[1]})
    with pytest.raises(APIException, match="400|registry"):
        admin.delete("/api/v1/checkpoints", body={"checkpoint_uuids": uuids[1:]})
    admin.delete("/api/v1/checkpoints", body={"checkpoint_uuids": uuids[:1]})
    assert admin.get(f"/api/v1/checkpoints/{uuids[0]}")["checkpoint"]["state"] == "DELETED"
    assert not os.path.exists(os.path.join(ckdir, uuids[0]))
