set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
rocminfo | grep -m3 -E "gfx|Marketing" > gpurun_out/r1_info.txt 2>&1 || true
timeout -k 10 400 python -m pytest tests/test_ops_gpu.py -x -q -m gpu > gpurun_out/r1_pytest.txt 2>&1
echo "pytest rc=$?" >> gpurun_out/r1_pytest.txt
timeout -k 10 300 python tools/probe_resnet.py --bn fused --steps 20 > gpurun_out/r1_probe_fused.txt 2>&1 && \
timeout -k 10 300 python tools/probe_resnet.py --bn torch --opt torch --dtype amp --steps 20 > gpurun_out/r1_probe_torch.txt 2>&1
echo done
