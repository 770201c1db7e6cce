cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=3 step fngrad timeout -k 10 300 python -u tools/diag/fieldn_grad_check.py
TAILN=20 step fnd5 timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fieldn.py
