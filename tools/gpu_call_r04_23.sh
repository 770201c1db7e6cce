cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
export SECT=1 FUSED_ONLY=1
TAILN=3 step fnprof timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/fnprof -o run -- python3 -u tools/diag/fieldn_train_time.py
f=$(ls $O/fnprof/*/run_kernel_stats.csv 2>/dev/null | head -1); [ -z "$f" ] && f=$(find $O/fnprof -name '*kernel_stats.csv' | head -1); cut -d, -f1-5 "$f" | head -25
