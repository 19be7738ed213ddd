set -o pipefail
OUT=gpurun_out/tailmap; mkdir -p $OUT
timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/c3.json 2> $OUT/c3.err && python3 -c "
import json; d=json.load(open('$OUT/c3.json')); k=d['roofline']['kernels']
print('C3', round(d['value'],1), 'wta', round(k['wta']['avg_ms'],4), round(k['wta']['tflops'],2), 'ahtw', round(k['ahtw']['avg_ms'],4), round(k['ahtw']['tflops'],2))" || exit 1
timeout -k 10 400 python -u -m pytest tests/test_gpu_c3.py tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "c3 or tile or narrow or block" > $OUT/tests.log 2>&1 && tail -1 $OUT/tests.log || { tail -20 $OUT/tests.log; exit 1; }
