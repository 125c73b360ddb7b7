"""Shipped TunableOp results (ops/gemm_tuning.py): merging tuning runs, CPU no-op."""
from determined_clone_amd.ops import gemm_tuning


def test_merge_unions_rows_and_keeps_validators(tmp_path):
    a = tmp_path / "a.csv"
    b = tmp_path / "b.csv"
    a.write_text("Validator,PT_VERSION,2.10.0\nValidator,GCN_ARCH_NAME,gfx950:sramecc+:xnack-\n"
                 "GemmTunableOp_BFloat16_NT,nt_1024_4096_1024,Gemm_Hipblaslt_1,0.1\n")
    b.write_text("Validator,PT_VERSION,2.10.0\n"
                 "GemmTunableOp_BFloat16_NT,nt_1024_4096_1024,Gemm_Hipblaslt_7,0.05\n"
                 "GemmTunableOp_BFloat16_TN,tn_64_64_32768,Gemm_Rocblas_3,0.02\n")
    out = tmp_path / "tuned" / "gemm.csv"
    assert gemm_tuning.merge([str(a), str(b)], str(out)) == 2
    lines = out.read_text().splitlines()
    assert lines[0].startswith("Validator,GCN_ARCH_NAME") and lines[1].startswith("Validator,PT_VERSION")
    assert "GemmTunableOp_BFloat16_NT,nt_1024_4096_1024,Gemm_Hipblaslt_7,0.05" in lines  # later run wins
    assert len(lines) == 4
    # merging into an existing file keeps its rows
    c = tmp_path / "c.csv"
    c.write_text("GemmTunableOp_float_NN,nn_8_8_8,Default,0.0\n")
    assert gemm_tuning.merge([str(c)], str(out)) == 3


def test_enable_is_a_noop_without_gpu(monkeypatch):
    import torch

    monkeypatch.setattr(torch.cuda, "is_available", lambda: False)
    monkeypatch.setitem(gemm_tuning._state, "path", None)
    assert gemm_tuning.enable() is False


def _validator():
    import importlib.util
    import os

    path = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tools",
                        "validate_tuned_gemms.py")
    spec = importlib.util.spec_from_file_location("validate_tuned_gemms", path)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    return mod


def test_validator_operands_reproduce_each_rows_layout():
    """tools/validate_tuned_gemms.py builds, for every shipped row, torch operands whose ``L @ R``
    is that row's column-major GEMM: shapes and leading dimensions as in the key."""
    import torch

    v = _validator()
    g = torch.Generator().manual_seed(0)
    n = 0
    for line in open(gemm_tuning.RESULTS):
        r = v.parse(line)
        if r is None or max(r["m"] * r["n"], r["k"] * r["n"], r["m"] * r["k"]) > 2e7:
            continue  # (large rows: same code path, too big for a CPU test)
        L, R = v.operands(r, g, "cpu")
        assert L.shape == (r["n"], r["k"]) and R.shape == (r["k"], r["m"])
        assert R.stride() == ((r["lda"], 1) if r["ta"] == "n" else (1, r["lda"]))
        assert L.stride() == ((r["ldb"], 1) if r["tb"] == "n" else (1, r["ldb"]))
        n += 1
    assert n > 20
    assert v.parse("Validator,PT_VERSION,2.10.0") is None
