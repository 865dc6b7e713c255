# A/B: every context with a high-priority exchange stream (FA_COMM_ALWAYS=1, up to round 5) against only
# rs contexts (now): north-star bench main line, alternating, after one warm-up process.
set -o pipefail
O=gpurun_out/${1:-r05s30}; mkdir -p $O
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary --no-live-pmc"
$B > $O/warm.json 2>$O/err || exit $?
for i in 1 2 3; do
    FA_COMM_ALWAYS=1 $B > $O/old$i.json 2>>$O/err || exit $?
    $B > $O/new$i.json 2>>$O/err || exit $?
done
for f in warm old1 new1 old2 new2 old3 new3; do python -c "import json;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['roofline']['kernel_ms_avg'],d['roofline']['frac'])"; done
