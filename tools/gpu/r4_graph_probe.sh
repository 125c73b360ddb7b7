#!/bin/bash
# HIP-graph vs eager, per activation / gradient, with MIOpen convolutions and without
set -o pipefail
mkdir -p gpurun_out
python -c "from determined_clone_amd.ops import _ext; print(_ext.load().__file__)" &&
DCA_CONV_DEBUG=1 timeout -k 10 240 python -u tools/probe_graph_miopen.py > gpurun_out/graph_probe_miopen.txt 2>&1 &&
timeout -k 10 240 python -u tools/probe_graph_miopen.py --no-miopen > gpurun_out/graph_probe_native.txt 2>&1
rc=$?
grep -E "first divergent|<==" gpurun_out/graph_probe_miopen.txt | head -30; grep "first divergent" gpurun_out/graph_probe_native.txt
exit $rc
