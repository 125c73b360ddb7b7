"""Which hipBLASLt epilogue configurations have gfx950 kernels in this library build (bf16 GEMMs,
fp32 accumulate): one JSON line per (epilogue, transposes, bias type, aux type, pointers set)."""
import itertools
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch  # noqa: E402

from determined_clone_amd.ops import _ext  # noqa: E402

EPI = {"DEFAULT": 1, "BIAS": 4, "GELU": 32, "GELU_BIAS": 36, "GELU_AUX": 160, "GELU_AUX_BIAS": 164,
       "DGELU": 192, "DGELU_BGRAD": 208, "BGRADA": 256, "BGRADB": 512}
R32F, R16BF = 0, 14  # hipDataType


def main():
    C = _ext.load()
    torch.zeros(1, device="cuda")
    for (name, e), (ta, tb), bt, at, ptrs in itertools.product(
            EPI.items(), ((True, False), (False, False), (False, True)), (-1, R32F, R16BF), (-1, R16BF, R32F),
            (False, True)):
        n = C.lt_probe(e, 4096, 32768, 1024, ta, tb, bt, at, ptrs)
        print(json.dumps({"epi": name, "ta": ta, "tb": tb, "bias_t": bt, "aux_t": at, "ptrs": ptrs, "algos": n}),
              flush=True)


if __name__ == "__main__":
    main()
