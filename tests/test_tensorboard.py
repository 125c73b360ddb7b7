"""TF event files: native writer -> native reader -> tensorboard task HTTP API."""
import json
import threading
import urllib.request

from determined_clone_amd import tensorboard
from determined_clone_amd.exec import tensorboard as tb_task


def test_event_roundtrip_and_server(tmp_path):
    w = tensorboard.MetricWriter(str(tmp_path / "trial" / "1"))
    for step in range(1, 4):
        w.on_metrics("training", step, {"loss": 1.0 / step, "note": "ignored"})
    w.on_metrics("validation", 3, {"acc": 0.5})
    w.close()
    runs = tensorboard.read_scalars(str(tmp_path))
    (run, tags), = runs.items()
    loss_tag = next(t for t in tags if t.endswith("loss"))
    assert [s for s, _, _ in tags[loss_tag]] == [1, 2, 3]
    assert abs(tags[loss_tag][-1][2] - 1 / 3) < 1e-6
    srv = tb_task.make_server({"exp": str(tmp_path)}, host="127.0.0.1")
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    base = f"http://127.0.0.1:{srv.server_address[1]}"
    listing = json.load(urllib.request.urlopen(base + "/data/runs"))
    r = next(iter(listing))
    data = json.load(urllib.request.urlopen(f"{base}/data/scalars?run={r}&tag={loss_tag}"))
    assert [d[1] for d in data] == [1, 2, 3]
    assert b"Scalars" in urllib.request.urlopen(base + "/").read()
    srv.shutdown()
