#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_dist_dopri5.py tests/test_gpu_dopri5.py -q --timeout 400 --timeout-method thread > $O/r03l_tests.log 2>&1
rc=$?; echo "tests rc=$rc"; tail -3 $O/r03l_tests.log
[ $rc -le 1 ] || exit $rc
timeout -k 10 300 python -u -c "
import bench, torch, json, numpy as np
import fet_ode_amd as F
dev = torch.device('cuda:0')
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5)
sd = {k: v.clone() for k, v in m.state_dict().items()}
y0 = bench.lv_y0(4096, 0).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
for mode in (0, 1):
    F._lib.load().fetode_resident_launch_mode(mode)
    r = bench.lv_dopri5_rate(sd, y0, t, reps=5)
    print('coop', mode, json.dumps({k: r[k] for k in ('ms_per_solve', 'attempts', 'nfev')}))
" > $O/r03l_dp5.log 2>&1
echo "dp5 rc=$?"; grep coop $O/r03l_dp5.log
