set -e
export TMPDIR=/tmp
tools/gpu_run.sh s3/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
tools/gpu_run.sh s3/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
tools/gpu_run.sh s3/bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
tools/gpu_run.sh s3/slot_small 200 python tools/slot_probe.py --small
for c in 4 5; do
  tools/gpu_run.sh s3/fetch$c 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s3/fetch$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
  tools/gpu_run.sh s3/write$c 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/s3/write$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
done
tools/gpu_run.sh s3/sweep5_bpc 300 python tools/sweep.py --config 5 --geoms "64,1,9" --bpc 1,2,3,4 --orders=-1,0 --rounds 3 --launches 10
