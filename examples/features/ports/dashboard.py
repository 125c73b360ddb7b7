"""A trial that serves a small HTTP "dashboard" on a task port while it trains, reached from the
user's machine through the master: ``det e create ports.yaml . -p 8265`` (the reference's
features/ports example does the same with a Ray head node; Ray is not in this image).

The dashboard reports the latest training step and loss; the trial trains a toy regression
with the Core API for ``hyperparameters.steps`` steps and then keeps serving for
``hyperparameters.linger_s`` seconds (so a tunnel can still be opened) unless preempted."""
import json
import os
import threading
import time
from http.server import BaseHTTPRequestHandler, ThreadingHTTPServer

import torch

import determined_clone_amd as det
from determined_clone_amd import core

STATE = {"step": 0, "loss": None}


class Dashboard(BaseHTTPRequestHandler):
    def log_message(self, *a):
        pass

    def do_GET(self):
        body = json.dumps(dict(STATE, task=os.environ.get("DET_TASK_ID"))).encode()
        self.send_response(200)
        self.send_header("Content-Type", "application/json")
        self.send_header("Content-Length", str(len(body)))
        self.end_headers()
        self.wfile.write(body)


def main(ctx: core.Context) -> None:
    info = det.get_cluster_info()
    hp = info.trial.hparams if info is not None else {"steps": 50, "linger_s": 0}
    port = int(os.environ.get("DASHBOARD_PORT", "8265"))
    srv = ThreadingHTTPServer(("0.0.0.0", port), Dashboard)
    threading.Thread(target=srv.serve_forever, daemon=True).start()
    print(f"dashboard on port {port}", flush=True)
    torch.manual_seed(0)
    w = torch.zeros(4, requires_grad=True)
    x = torch.randn(256, 4)
    y = x @ torch.tensor([1.0, -2.0, 0.5, 3.0])
    opt = torch.optim.SGD([w], lr=0.1)
    for step in range(1, int(hp["steps"]) + 1):
        loss = ((x @ w - y) ** 2).mean()
        opt.zero_grad()
        loss.backward()
        opt.step()
        STATE.update(step=step, loss=float(loss))
        if step % 10 == 0:
            ctx.train.report_training_metrics(steps_completed=step, metrics={"loss": float(loss)})
        if ctx.preempt.should_preempt():
            return
    ctx.train.report_validation_metrics(steps_completed=int(hp["steps"]), metrics={"loss": float(loss)})
    deadline = time.time() + float(hp.get("linger_s", 0))
    while time.time() < deadline and not ctx.preempt.should_preempt():
        time.sleep(0.5)
    srv.shutdown()


if __name__ == "__main__":
    with core.init() as ctx:
        main(ctx)
