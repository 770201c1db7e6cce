cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
rm -f gpurun_out/head_sd.pt
TAILN=1 step h4 env TAG=v4 timeout -k 10 120 python -u tools/diag/mnist_head_time.py
TAILN=1 step h1 env TAG=v1 FETODE_WIDE_V=1 timeout -k 10 120 python -u tools/diag/mnist_head_time.py
python -c "
import torch; b=torch.load('gpurun_out/head_v1.pt'); c=torch.load('gpurun_out/head_v4.pt')
print('bitwise v4/v1', torch.equal(c,b))"

