cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=45 step hostp timeout -k 10 300 python -u tools/diag/host_path_profile.py
