#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dopri5.py tests/test_gpu_ecg.py tests/test_gpu_dist_dopri5.py tests/test_gpu_ett.py tests/test_gpu_lv.py -q --timeout 400 --timeout-method thread > $O/r03m_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r03m_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "
import bench, torch, json
r = bench.ett_dopri5_rate(torch.device('cuda:0'))
print('ett', json.dumps({k: r[k] for k in ('ms_per_batch', 'attempts', 'nfev', 'field_eval_ms', 'host_share')}))
" > $O/r03m_ett.log 2>&1
echo "ett rc=$?"; grep "^ett" $O/r03m_ett.log
