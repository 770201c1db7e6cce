cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=30 step newtests2 timeout -k 10 600 python -u -m pytest -q --timeout 300 --timeout-method thread tests/test_gpu_dist_wide_dopri5.py "tests/test_gpu_grad.py::test_small_batch_tape_matches_v4"
TAILN=12 step ettnan timeout -k 10 200 python -u tools/diag/ett_nan2.py
step ettprof env B=8192 P=24 TSCALE=0.05 ITERS=1 timeout -k 10 400 rocprofv3 --kernel-trace --stats -d $O/ettprof -o run --output-format csv -- python3 tools/diag/ett_dopri5_train.py
f=$(find $O/ettprof -name '*kernel_stats.csv' | head -1); cp "$f" $O/r04_ett_dopri5_train_kernel_stats.csv; rm -rf $O/ettprof
head -15 $O/r04_ett_dopri5_train_kernel_stats.csv | cut -c1-200
