"""tools/api_load_test.py (the reference's k6 API load test, performance/src/api_performance_tests.ts)
against an in-process master: seeding, ramping virtual users, thresholds and reports."""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "tools"))

import api_load_test as lt  # noqa: E402

from determined_clone_amd.master import Master, MasterServer  # noqa: E402


def test_stage_parsing_and_ramp():
    st = lt.parse_stages("2s:4,1m:4,500ms:0".replace("500ms", "0.5s"))
    assert st == [(2.0, 4), (60.0, 4), (0.5, 0)]
    assert lt.target_at(st, 0.0) == 0 and lt.target_at(st, 1.0) == 2 and lt.target_at(st, 30) == 4
    assert lt.target_at(st, 62.25) == 2 and lt.target_at(st, 63.0) == -1


def test_load_run_against_seeded_master(tmp_path, capsys):
    m = Master(str(tmp_path / "m.db"))
    srv = MasterServer(m, "127.0.0.1", 0).start()
    try:
        rc = lt.main(["-m", m.master_url, "--seed", "--stages", "1s:4,2s:4,0.5s:0", "--think-s", "0.05",
                      "--junit", str(tmp_path / "r.xml"), "--json", str(tmp_path / "r.json")])
        out = capsys.readouterr().out
        r = json.load(open(tmp_path / "r.json"))
        assert r["failed"] == 0, {g: d.get("error") for g, d in r["groups"].items() if d["failed"]}
        assert rc == 0, out
        assert r["peak_vus"] == 4 and r["requests"] > 100
        for g in ("get experiment batches", "get model version", "get task logs", "get trial workloads",
                  "get experiment trials snapshot", "login"):
            assert r["groups"][g]["count"] > 0, g
        assert "PASS http_req_failed" in out
        assert 'failures="0"' in open(tmp_path / "r.xml").read()
    finally:
        srv.stop()
