cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=3 step wbt timeout -k 10 120 python -u tools/diag/wide_bwd_time.py
TAILN=20 step t6 timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_dist_train.py "tests/test_gpu_grad.py::test_small_batch_tape_matches_v4" tests/test_gpu_dist_wide_dopri5.py tests/test_gpu_ett.py
TAILN=4 step ett_d5_train8k env B=8192 P=24 TSCALE=0.05 ITERS=1 timeout -k 10 300 python -u tools/diag/ett_dopri5_train.py
