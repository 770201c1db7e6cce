cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=60 step tgc env KIND=kanfet timeout -k 10 300 python -u tools/diag/tape_grad_check.py
TAILN=12 step ettnan timeout -k 10 200 python -u tools/diag/ett_nan2.py
TAILN=4 step ett_d5_train8k env B=8192 P=24 TSCALE=0.05 ITERS=1 timeout -k 10 300 python -u tools/diag/ett_dopri5_train.py
TAILN=30 step d5tests timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dopri5_train.py tests/test_gpu_ett.py tests/test_gpu_ecg.py tests/test_gpu_dist_train.py
