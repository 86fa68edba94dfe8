#!/bin/bash
# round 5: full pass of the tree after the LZ77 writer, the inflate rework and the deep column kernels -- GPU tests, smoke,
# the two PMC traffic passes of the same bench command (device chain only)
set -o pipefail
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/${RUN:-r05ak}
mkdir -p $O
cd $R
timeout -k 10 700 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider \
  > $O/pytest_gpu.log 2>&1 || { tail -n 40 $O/pytest_gpu.log; exit 1; }
tail -n 1 $O/pytest_gpu.log
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -n 20 $O/smoke.log; exit 1; }
tail -n 1 $O/smoke.log
timeout -k 10 500 python -u bench.py > $O/bench.json 2> $O/bench.err || { tail -n 30 $O/bench.err; exit 1; }
python -c "import json;d=json.load(open('$O/bench.json'));print('bench', d['ms_per_step'], d['value'], d['roofline']['frac'], d.get('from_files_config2',{}).get('steps_4_7_s'), d.get('config3_1gpu',{}).get('ms_per_step'))"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 3 --warmup 1 --no-cpu-baseline --no-files-baseline --no-files-config2 --config3-steps 0"
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/stats -- python3 $B > $O/stats.log 2>&1 || { tail -n 20 $O/stats.log; exit 1; }
echo stats ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc FETCH_SIZE -d $O/pmc_fetch -- python3 $B > $O/pmc_fetch.log 2>&1 || { tail -n 20 $O/pmc_fetch.log; exit 1; }
echo pmc fetch ok
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv --pmc WRITE_SIZE -d $O/pmc_write -- python3 $B > $O/pmc_write.log 2>&1 || { tail -n 20 $O/pmc_write.log; exit 1; }
echo pmc write ok
