"""Shipped MIOpen DB / kernel cache wiring (ops/miopen_db.py)."""
import os

from determined_clone_amd.ops import miopen_db


def test_shipped_files_exist_and_configure_respects_env():
    db, cache = miopen_db.shipped_dirs()
    assert any(f.endswith(".ufdb.txt") for f in os.listdir(db)), "find DB not shipped"
    assert any(f.endswith(".ukdb") for f in os.listdir(cache)), "kernel cache not shipped"
    env = {}
    got = miopen_db.configure(env)
    assert got == {"MIOPEN_USER_DB_PATH": db, "MIOPEN_CUSTOM_CACHE_DIR": cache}
    env = {"MIOPEN_USER_DB_PATH": "/x", "MIOPEN_CUSTOM_CACHE_DIR": "/y"}
    assert miopen_db.configure(env) == env  # an explicit choice wins


def test_task_dirs_seeded_once_and_kept(tmp_path):
    db, cache = miopen_db.task_dirs(str(tmp_path))
    assert sorted(os.listdir(db)) == sorted(os.listdir(miopen_db.shipped_dirs()[0]))
    (tmp_path / "miopen" / "cache" / "extra.ukdb").write_text("x")
    db2, cache2 = miopen_db.task_dirs(str(tmp_path))
    assert (db2, cache2) == (db, cache) and os.path.exists(os.path.join(cache2, "extra.ukdb"))
