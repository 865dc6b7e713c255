set -o pipefail
O=gpurun_out/r05s26; mkdir -p $O
B="timeout -k 10 200 python bench.py --no-cpu-baseline --no-secondary"
$B --no-live-pmc > $O/a1.json 2>$O/err && \
$B --no-live-pmc > $O/a2.json 2>>$O/err && \
timeout -k 10 120 python tools/order_effect.py 129 alloc-only 2>>$O/err && sleep 12 && \
$B --no-live-pmc > $O/a3.json 2>>$O/err && \
$B > $O/a4.json 2>>$O/err && \
$B --no-live-pmc > $O/a5.json 2>>$O/err
rc=$?
for f in a1 a2 a3 a4 a5; do python -c "import json,sys;d=json.loads(open('$O/$f.json').read().strip().splitlines()[-1]);print('$f',d['value'],d['roofline']['kernel_ms_avg'],d['roofline']['frac'])"; done
exit $rc
