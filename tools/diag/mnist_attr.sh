cd /root/repo; export TMPDIR=/tmp
for v in base:libfetode.so nomfma:libfetode_v1.so nofeat:libfetode_v2.so neither:libfetode_v3.so; do n=${v%%:*}
FETODE_LIB=$PWD/fet-ode_amd/${v#*:} timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/mnq_$n -o run --output-format csv -- python3 tools/diag/mnist_prof.py > gpurun_out/mnq_$n.log 2>&1 || exit 3
echo "== $n: $(python tools/diag/kstats.py gpurun_out/mnq_$n 6 | grep wide_fwd)"; done
