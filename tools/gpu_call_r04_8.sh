cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=10 step widetests timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_wide.py tests/test_gpu_ett.py tests/test_gpu_ecg.py
TAILN=3 step wbt2 timeout -k 10 120 python -u tools/diag/wide_bwd_time.py
TAILN=3 step wbt1 env FETODE_FERRO_BWD_OGW=1 timeout -k 10 120 python -u tools/diag/wide_bwd_time.py
TAILN=3 step wbt4 env FETODE_FERRO_BWD_OGW=4 timeout -k 10 120 python -u tools/diag/wide_bwd_time.py
