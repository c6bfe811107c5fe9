set -e
tools/gpu_run.sh s1/e2e2 300 python tools/bench_e2e.py --config 2
tools/gpu_run.sh s1/hbm_probe 200 python tools/hbm_probe.py
tools/gpu_run.sh s1/build_v6 200 python tools/bench_build.py --family 6
tools/gpu_run.sh s1/build_64 200 python tools/bench_build.py --payload 64
tools/gpu_run.sh s1/smoke 120 python -c "import __graft_entry__ as g; g.smoke()"
