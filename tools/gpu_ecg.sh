cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_ecg.py > gpurun_out/ecg.log 2>&1
rc=$?; echo "ecg rc=$rc"; grep -E "PASS|FAIL|Error|assert" gpurun_out/ecg.log | head -30
