set -u
OUT=gpurun_out/r02s06; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_ctx_layouts.py tests/test_gpu_parity.py tests/test_e2e_aggregator.py -x -q -rfs --timeout 240 --timeout-method thread > $OUT/pytest.log 2>&1; rc=$?; tail -8 $OUT/pytest.log; [ $rc -le 1 ] || exit $rc
timeout -k 10 400 python bench.py --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err; rc=$?; python -c "
import json;d=json.load(open('$OUT/bench.json'));print(d['value'],d['roofline']['frac'],d['roofline']['kernel_ms_avg']);[print(k,v.get('kernel_ms_avg'),v.get('frac')) for k,v in d['secondary'].items()]"
exit $rc
