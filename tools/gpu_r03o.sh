#!/bin/bash
cd "$(dirname "$0")/.."
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -c "
import bench, torch, json, numpy as np
import fet_ode_amd as F
dev = torch.device('cuda:0')
torch.manual_seed(0)
m = F.KANFET([2, 10, 2], grid_size=5).to(dev)
y0 = bench.lv_y0(4096, 0).to(dev)
t = torch.tensor(np.linspace(0, 3.5, 35))
for rep in range(2):
    r = bench.train_rate(m, y0, t, 50, 5, 1)
    print('train', json.dumps({'value': r['value'], 'ms': r['ms_per_iter'], 'eager': r['eager']['value'], 'eager_ms': r['eager']['ms_per_iter']}))
" > $O/r03o_train.log 2>&1
echo "train rc=$?"; grep -E "^train|Error" $O/r03o_train.log
