set -e
O=gpurun_out/r02t; mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_depth16.py tests/test_gpu_streamed.py tests/test_gpu_sharded.py tests/test_gpu_e2e.py -x -q --timeout 300 --timeout-method thread > $O/pytest.log 2>&1
echo "pytest: $(tail -1 $O/pytest.log)"
timeout -k 10 200 python -u bench.py --no-cpu-baseline > $O/bench.json 2> $O/bench.err
python3 -c "import json;d=json.load(open('$O/bench.json'));print(round(d['value']), d['ms_per_step'], d['stages_ms'])"
