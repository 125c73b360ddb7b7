"""Shipped convolution-chooser decisions (ops/tuned/conv_choices_gfx950.json) and the multi-rank
policy of ops/conv.py ``_choose`` (gloo, 2 ranks)."""
import json
import os
import socket
import tempfile

import torch
import torch.multiprocessing as mp

from determined_clone_amd.ops import conv


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_dump_load_round_trip(tmp_path):
    saved = dict(conv._CHOICE)
    try:
        conv._CHOICE.clear()
        key = ("dgrad", (8, 256, 56, 56), 64, 1, torch.bfloat16)
        conv._CHOICE[key] = 1
        conv._CHOICE[("wgrad", (8, 64, 56, 56), (64, 64, 3, 3), 1, 1)] = 0
        p = str(tmp_path / "c.json")
        conv.dump_choices(p, "test")
        data = json.load(open(p))
        assert data["device"] == "test" and len(data["choices"]) == 2
        conv._CHOICE.clear()
        assert conv.load_choices(p) == 2
        assert conv._CHOICE[key] == 1
        # a shipped decision is used without timing
        before = conv.TIMINGS
        assert conv._choose(key, (lambda: None, lambda: None)) == 1 and conv.TIMINGS == before
    finally:
        conv._CHOICE.clear()
        conv._CHOICE.update(saved)


def test_shipped_file_is_well_formed():
    path = conv._SHIPPED_PATH
    if not os.path.exists(path):
        return
    data = json.load(open(path))
    for e in data["choices"]:
        key = conv._key_from_json(e["key"])
        assert key[0] in ("fwd", "dgrad", "wgrad", "fwd1x1+bn") and e["choice"] in (0, 1)


def _worker(rank, world, port, out, dist_tune):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port)})
    torch.distributed.init_process_group("gloo", rank=rank, world_size=world)
    conv._CHOICE.clear()
    conv.AUTOTUNE_DIST = dist_tune
    # rank-dependent timings: rank 0 finds candidate 1 fastest, rank 1 candidate 0
    conv._time_us = lambda fn: {(0, 0): 9.0, (0, 1): 1.0, (1, 0): 1.0, (1, 1): 9.0}[(rank, fn())]
    picks = [conv._choose(("fwd", (4, 64, 8, 8), 64, 1, torch.bfloat16), (lambda: 0, lambda: 1)),
             conv._choose(("dgrad", (4, 64, 8, 8), 64, 1, torch.bfloat16), (lambda: 0, lambda: 1))]
    json.dump({"picks": picks, "timings": conv.TIMINGS}, open(os.path.join(out, f"r{rank}.json"), "w"))
    torch.distributed.destroy_process_group()


def test_ranks_make_identical_choices():
    for dist_tune, want in ((False, [0, 0]), (True, [1, 1])):
        with tempfile.TemporaryDirectory() as d:
            mp.spawn(_worker, args=(2, _free_port(), d, dist_tune), nprocs=2, join=True)
            r = [json.load(open(os.path.join(d, f"r{i}.json"))) for i in range(2)]
        assert r[0]["picks"] == r[1]["picks"] == want
        # default multi-rank policy: unseen shapes are not timed at all
        assert (r[0]["timings"] == 0) == (not dist_tune)
