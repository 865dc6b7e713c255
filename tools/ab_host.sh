# The north star from C++ alone (bin/fa_bench: libfa's streams, no torch stream pool) against bench.py's
# main line (torch streams), alternating on one box after a warm-up process.
set -o pipefail
O=gpurun_out/${1:-r05s33}; mkdir -p $O
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-live-pmc"
F="timeout -k 10 120 multihop-federeated-split-learning_amd/bin/fa_bench --workload northstar --steps 20 --warmup 5"
$B > $O/warm.json 2>$O/err || exit $?
for i in 1 2 3; do
    $F > $O/cpp$i.json 2>>$O/err || exit $?
    $B > $O/py$i.json 2>>$O/err || exit $?
done
for i in 1 2 3; do tail -1 $O/cpp$i.json | cut -c1-400; python -c "import json;d=json.loads(open('$O/py$i.json').read().strip().splitlines()[-1]);print('py',d['value'],d['roofline']['kernel_ms_avg'],d['roofline']['frac'])"; done
