cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=6 step fntests timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_fieldn_train.py tests/test_gpu_fieldn.py tests/test_gpu_grad.py
TAILN=6 step fnlds timeout -k 10 400 python -u tools/diag/fieldn_train_time.py
export SECT=1 FUSED_ONLY=1
TAILN=2 step fnprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fnprof -o run -- python3 -u tools/diag/fieldn_train_time.py
