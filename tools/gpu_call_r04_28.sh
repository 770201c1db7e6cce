cd $GRAFT_REPO_ROOT
O=gpurun_out; mkdir -p $O
export TMPDIR=/tmp
step() { local name=$1; shift; "$@" > $O/$name.log 2>&1; local rc=$?; echo "$name rc=$rc"; tail -${TAILN:-15} $O/$name.log; [ $rc -le 1 ] || exit $rc; return 0; }
TAILN=4 step fntests timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu
export SECT=23
TAILN=5 step fnlds timeout -k 10 400 python -u tools/diag/fieldn_train_time.py
unset SECT
TAILN=1 step bench timeout -k 10 600 python bench.py
tail -1 $O/bench.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['value'], d['strong_proxy'])"
