"""AddressSanitizer(+UBSan) and ThreadSanitizer builds of the native runtime, the counterpart of
the reference master's ``go test -race``:

* the scheduler module (native/scheduler.cpp) is loaded into a Python whose allocator is the
  sanitizer runtime (LD_PRELOAD) and driven from 8 Python threads at once -- the master calls
  ``Scheduler.schedule`` with the GIL released -- over every policy / fitting method, plus
  ``find_fit`` and the KFD topology reader on a fake sysfs tree;
* the pidwatch launcher (native/pidwatch.cpp) runs its success and teardown scenarios.

Any sanitizer report fails the test (halt_on_error, exit code 66). CPU only."""
import os
import subprocess
import sys
import textwrap

import pytest

from determined_clone_amd.native import build

KINDS = ["asan", "tsan"]
ENV = {
    "asan": {"ASAN_OPTIONS": "detect_leaks=0:halt_on_error=1:exitcode=66:abort_on_error=0",
             "UBSAN_OPTIONS": "halt_on_error=1:exitcode=66:print_stacktrace=1"},
    "tsan": {"TSAN_OPTIONS": "halt_on_error=1:exitcode=66:report_signal_unsafe=0"},
}

DRIVER = textwrap.dedent('''
    import importlib.machinery, importlib.util, os, random, sys, threading
    path, sysfs = sys.argv[1], sys.argv[2]
    loader = importlib.machinery.ExtensionFileLoader("_native", path)
    spec = importlib.util.spec_from_file_location("_native", path, loader=loader)
    N = importlib.util.module_from_spec(spec)
    loader.exec_module(N)

    def agent(aid, slots, rng):
        a = N.Agent(); a.id = aid; a.num_slots = slots; a.pool = "default"
        a.slot_owner = ["" if rng.random() < 0.7 else f"x{rng.randrange(4)}" for _ in range(slots)]
        a.slot_enabled = [rng.random() < 0.95 for _ in range(slots)]
        return a

    def req(aid, rng):
        r = N.Request(); r.alloc_id = aid; r.job_id = f"job{rng.randrange(5)}"
        r.slots = rng.choice([0, 1, 1, 2, 4, 8, 16]); r.priority = rng.randrange(1, 99)
        r.weight = rng.choice([0.5, 1.0, 3.0]); r.submit_time = rng.random()
        r.preemptible = rng.random() < 0.8; r.blocked_agents = [f"a{rng.randrange(6)}"] if rng.random() < 0.2 else []
        return r

    def run(aid, rng):
        r = N.Running(); r.alloc_id = aid; r.job_id = f"job{rng.randrange(5)}"
        r.slots = rng.choice([1, 2, 4]); r.priority = rng.randrange(1, 99); r.start_time = rng.random()
        r.preemptible = rng.random() < 0.8
        return r

    shared = {p: N.Scheduler(p, f, True) for p, f in (("priority", "best"), ("fair_share", "worst"),
                                                     ("round_robin", "best"))}
    errors = []

    def work(k):
        rng = random.Random(k)
        try:
            for i in range(150):
                agents = [agent(f"a{j}", rng.choice([4, 8]), rng) for j in range(rng.randrange(1, 6))]
                pend = [req(f"t{k}-{i}-{j}", rng) for j in range(rng.randrange(0, 14))]
                runn = [run(f"r{k}-{i}-{j}", rng) for j in range(rng.randrange(0, 6))]
                for s in shared.values():
                    d = s.schedule(agents, pend, runn)
                    used = {}
                    for alloc, places in d.start:
                        for p in places:
                            for sl in p.slots:
                                key = (p.agent_id, sl)
                                assert key not in used, f"slot {key} given twice"
                                used[key] = alloc
                N.find_fit(pend[0], agents, "best") if pend else None
                if i % 25 == 0:
                    N.detect_kfd_gpus(sysfs)
        except Exception as e:  # noqa: BLE001
            errors.append(repr(e))

    ts = [threading.Thread(target=work, args=(k,)) for k in range(8)]
    [t.start() for t in ts]
    [t.join() for t in ts]
    assert not errors, errors
    print("driver ok")
''')


def _fake_sysfs(root):
    for node, props in (("0", "cpu_cores_count 8\nsimd_count 0\n"),
                        ("1", "simd_count 1024\ngfx_target_version 90500\nunique_id 1234\ndrm_render_minor 128\n")):
        d = os.path.join(root, node)
        os.makedirs(os.path.join(d, "mem_banks", "0"), exist_ok=True)
        with open(os.path.join(d, "properties"), "w") as f:
            f.write(props)
        with open(os.path.join(d, "gpu_id"), "w") as f:
            f.write("5" if node == "1" else "0")
        with open(os.path.join(d, "mem_banks", "0", "properties"), "w") as f:
            f.write("size_in_bytes 309237645312\n")


@pytest.fixture(scope="module", params=KINDS)
def sanitized(request):
    kind = request.param
    rt = build.sanitizer_runtime(kind)
    if not rt:
        pytest.skip(f"no {kind} runtime for this compiler")
    try:
        mod, pw = build.build_sanitized(kind)
    except RuntimeError as e:
        pytest.skip(str(e)[:500])
    return kind, rt, str(mod), str(pw)


def _env(kind, preload=None):
    env = dict(os.environ, **ENV[kind])
    if preload:
        env["LD_PRELOAD"] = preload
    return env


def _no_report(kind, stderr):
    for marker in ("ERROR: AddressSanitizer", "runtime error:", "WARNING: ThreadSanitizer",
                   "ERROR: ThreadSanitizer", "SUMMARY: UndefinedBehaviorSanitizer"):
        assert marker not in stderr, f"{kind} report:\n{stderr[-4000:]}"


def test_scheduler_from_many_python_threads(sanitized, tmp_path):
    kind, rt, mod, _ = sanitized
    sysfs = tmp_path / "topology"
    _fake_sysfs(str(sysfs))
    drv = tmp_path / "driver.py"
    drv.write_text(DRIVER)
    r = subprocess.run([sys.executable, str(drv), mod, str(sysfs)], env=_env(kind, rt),
                       capture_output=True, text=True, timeout=600)
    _no_report(kind, r.stderr)
    assert r.returncode == 0 and "driver ok" in r.stdout, r.stderr[-3000:]


def test_pidwatch_scenarios(sanitized, tmp_path):
    kind, _, _, pw = sanitized

    def launch(addr, workers):
        clients = " & ".join(f"{pw} client {addr} -- {w}" for w in workers)
        return [pw, "server", "--grace-period", "1", addr, str(len(workers)), "--", "bash", "-c",
                clients + " & wait"]

    ok = subprocess.run(launch(str(tmp_path / "a.sock"), ["true", "sleep 0.3"]), env=_env(kind),
                        capture_output=True, text=True, timeout=120)
    _no_report(kind, ok.stderr)
    assert ok.returncode == 0, ok.stderr[-2000:]
    bad = subprocess.run(launch(str(tmp_path / "b.sock"), ["sleep 30", "bash -c 'sleep 0.3; exit 3'"]),
                         env=_env(kind), capture_output=True, text=True, timeout=120)
    _no_report(kind, bad.stderr)
    assert bad.returncode == 70, bad.stderr[-2000:]
