cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
rm -f $O/wide_sd_*.pt
TAILN=2 step wf1 env TAG=fast timeout -k 10 120 python -u tools/diag/wide_fwd_time.py
TAILN=2 step wf0 env TAG=slow FETODE_WIDE_FASTF=0 timeout -k 10 120 python -u tools/diag/wide_fwd_time.py
TAILN=2 step wf2 env TAG=fast2 timeout -k 10 120 python -u tools/diag/wide_fwd_time.py
python -c "
import torch
for s in ('64_128','128_64'):
    a=torch.load(f'gpurun_out/wide_fast_{s}.pt'); b=torch.load(f'gpurun_out/wide_slow_{s}.pt'); print(s, 'bitwise', torch.equal(a,b))"
