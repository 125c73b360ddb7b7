"""Every shipped TunableOp result computes the right numbers (tools/validate_tuned_gemms.py).

TunableOp keeps the fastest solution per shape and, unless told to, never compares its output
with anything; round 6 found a shipped hipBLASLt solution (ResNet-50's layer1 1x1 forward at
bs 1024) that was fastest because a fraction of its outputs were wrong
(profiles/round6_tuned_gemm_validation.txt). The validator replays the file in its own process
(TunableOp state is process-global) and checks each row against an fp32 reference."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_every_shipped_tuned_gemm_is_numerically_correct():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "validate_tuned_gemms.py")],
                         capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-2000:]
    rows = [json.loads(ln) for ln in out.stdout.splitlines() if ln.startswith("{")]
    summary = rows[-1]["summary"]
    assert summary["bad"] == [], summary
    checked = [r for r in rows[:-1] if "ok" in r]
    assert len(checked) >= 100 and all(r["ok"] for r in checked)
