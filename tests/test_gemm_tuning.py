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
