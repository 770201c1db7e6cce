cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=12 step pend timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dist_wide_dopri5.py tests/test_gpu_dist_train.py tests/test_gpu_grad.py tests/test_gpu_dist_models.py
TAILN=6 step ettd5 timeout -k 10 300 python -u tools/diag/ett_dopri5_train.py
