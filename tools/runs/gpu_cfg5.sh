set -e
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/cfg5
for s in 10000 50000; do
  timeout -k 10 400 python -u tools/bench_loci.py --samples $s --loci 734 --reps 2 --cpu-samples 200 > gpurun_out/cfg5/loci_$s.json 2> gpurun_out/cfg5/loci_$s.err
  python -c "import json; d=json.load(open('gpurun_out/cfg5/loci_$s.json')); print($s, d['device_ms'], d['host_prep_s'], d['end_to_end_s'])"
done
