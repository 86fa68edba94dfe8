set -e
O=gpurun_out/r02p; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
echo "pytest: $(tail -1 $O/pytest_gpu.log)"
timeout -k 10 200 python -u bench.py --depth-format q16 --no-cpu-baseline > $O/bench_q16.json 2> $O/bench_q16.err
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench_i32.json 2> $O/bench_i32.err
python3 -c "
import json
for f in ['q16','i32']:
    d=json.load(open('$O/bench_'+f+'.json')); print(f, round(d['value']), d['ms_per_step'], d['stages_ms'])"
