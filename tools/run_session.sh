#!/bin/bash
# One parameterised GPU-box runner for the recurring checks (it replaces the
# per-round tools/r0x_*.sh scripts, kept verbatim in
# profiles/run_scripts.bundle.txt).  Every GPU step runs under its own time
# limit through tools/gpu_run.sh, which stops the chain at a fault, abort or
# time-out; logs go to gpurun_out/<tag>/.
#
#   tools/run_session.sh <tag> <recipe> [<recipe> ...]
#
# recipes:
#   env       read-only box facts bearing on registered host memory (THP,
#             memlock, compaction, NUMA balancing)
#   suite     the product GPU suite (XCSUM_REG_TRACE on), smoke, the driver's
#             bench command
#   debug     the GPU suite on the bounds-checked build (libxudp_amd/debug,
#             built beforehand: make -C libxudp_amd debug)
#   benches   bench.py over its workloads, one summary line each
#             (BENCH_ARGS: '|'-separated argument lists to replace the default)
#   e2e       host-resident end-to-end rates (tools/bench_e2e.py)
#   ring      libxudp's TX loop on its anon_map UMEM (tests/c/umem_ring --bench)
#   crossover one host core running the reference's xudp_packet_udp
#             (tools/crossover.py)
#   iphdr     the header-only legs of libxudp's IPv4 TX call
#             (tools/iphdr_probe.py) and the build kernel's (tools/bench_build.py)
#   iphdr_pmc FETCH/WRITE/request counters of the header-only kernel, one
#             rocprofv3 pass per counter set and leg (tools/pmc_legs.py
#             summarises gpurun_out/<tag>/pmc)
#   build_pmc FETCH/WRITE/request counters of the IPv4 in-place build
#             (build_hdr_kernel through tools/bench_build.py)
#   profile   tools/profile_round.sh <tag>/profile (bench lines, kernel
#             stats, PMC summaries)
set -u
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
t="$1"; shift
mkdir -p "gpurun_out/$t"
P="python -u -m pytest tests -m gpu -x -q -s --timeout 300 --timeout-method thread"
DEFAULT_BENCHES="--config 2|--config 2 --layout umem|--config 3|--config 4|--config 5\
|--config 2 --flags inplace,iphdr_only|--config 2 --flags inplace,iphdr_only --layout umem\
|--config 2 --flags inplace,iphdr|--config 4 --flags inplace|--config 2 --flags verify"

env_facts() {
  echo "uname: $(uname -r)"
  echo "ulimit -l: $(ulimit -l)"
  for f in /sys/kernel/mm/transparent_hugepage/enabled \
           /sys/kernel/mm/transparent_hugepage/shmem_enabled \
           /sys/kernel/mm/transparent_hugepage/defrag \
           /proc/sys/vm/compact_unevictable_allowed \
           /proc/sys/kernel/numa_balancing \
           /sys/module/amdgpu/parameters/noretry \
           /sys/module/amdgpu/parameters/mtype_local; do
    [ -r "$f" ] && echo "$f: $(cat "$f" 2>/dev/null)"
  done
  grep -E 'thp_|compact_(migrate|stall|success)|pgmigrate' /proc/vmstat 2>/dev/null | tr '\n' ' '
  echo
}

for r in "$@"; do
  case "$r" in
  env)
    env_facts > "gpurun_out/$t/env.log" 2>&1 ;;
  suite)
    XCSUM_REG_TRACE=$PWD/gpurun_out/$t/regtrace.log tools/gpu_run.sh $t/pytest_gpu 900 $P &&
    tools/gpu_run.sh $t/smoke 200 python -c "import __graft_entry__ as g; g.smoke()" &&
    tools/gpu_run.sh $t/bench_driver_cmd 300 python bench.py --gpus 1 --steps 20 --warmup 5 \
      || exit $? ;;
  debug)
    XCSUM_LIB=$PWD/libxudp_amd/debug/libxcsum.so tools/gpu_run.sh $t/pytest_gpu_debug 900 $P \
      || exit $? ;;
  benches)
    IFS='|' read -ra lines <<< "${BENCH_ARGS:-$DEFAULT_BENCHES}"
    i=0
    for a in "${lines[@]}"; do
      i=$((i + 1))
      tools/gpu_run.sh $t/bench_$i 300 python -u bench.py --steps 100 --warmup 5 \
        --no-cpu-baseline $a || exit $?
      python3 - "gpurun_out/$t/bench_$i.log" "$a" >> "gpurun_out/$t/benches.txt" <<'PY'
import json, sys
rows = [l for l in open(sys.argv[1]) if l.startswith("{")]
if not rows:
    print(sys.argv[2], "| no line")
    raise SystemExit
d = json.loads(rows[-1]); r = d["roofline"]
print(sys.argv[2], "|", d["value"], "GiB/s |", d["kernel_ms"], "ms |", d["mpps"], "Mpps | frac",
      r["frac"], "| vs ceiling", r.get("frac_vs_ceiling"), "| order",
      d["config"].get("order_calibration"), "| parity", d.get("parity_ok"))
PY
    done ;;
  e2e)
    for a in "--config 2" "--config 2 --layout umem" "--config 4"; do
      tools/gpu_run.sh "$t/e2e_$(echo $a | tr ' -' '__')" 300 python -u tools/bench_e2e.py $a \
        --reps 5 || exit $?
    done ;;
  crossover)
    tools/gpu_run.sh $t/crossover 300 python -u tools/crossover.py || exit $? ;;
  ring)
    # libxudp's TX loop on its anon_map UMEM, every variant launched and with
    # 16 resident workgroups (tests/c/umem_ring.c)
    RING_RESIDENT_WG=16 XCSUM_RESIDENT_TRACE=1 tools/gpu_run.sh $t/ring_bench 400 \
      tests/c/umem_ring --bench 1,16,100,1024 || exit $? ;;
  iphdr)
    tools/gpu_run.sh $t/iphdr_probe 400 python -u tools/iphdr_probe.py --rounds 3 &&
    tools/gpu_run.sh $t/bench_build 300 python -u tools/bench_build.py \
      --modes inplace,inplace_sum,copy_aligned --reps 30 || exit $? ;;
  iphdr_pmc)
    mkdir -p gpurun_out/$t/pmc
    for lay in packed slots; do
      for leg in inplace out_only; do
        for pmc in FETCH_SIZE WRITE_SIZE \
                   "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
          tag=$(echo "$pmc" | cut -d' ' -f1)
          d=gpurun_out/$t/pmc/${lay}_${leg}_$tag
          # --warm 0 and one leg: every counted dispatch is that leg's
          timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $d -o run -- \
            python3 tools/iphdr_probe.py --layouts $lay --legs $leg --rounds 1 --reps 1 \
            --per 3 --warm 0 --no-ref > $d.log 2>&1
          rc=$?
          echo "pmc $lay $leg $tag rc=$rc"
          [ $rc -eq 0 ] || exit $rc
        done
      done
    done ;;
  build_pmc)
    # the IPv4 in-place build (build_hdr_kernel, tools/bench_build.py
    # inplace): FETCH/WRITE and the L2's memory-side requests, one pass each
    mkdir -p gpurun_out/$t/bpmc
    for pmc in FETCH_SIZE WRITE_SIZE \
               "TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
      tag=$(echo "$pmc" | cut -d' ' -f1)
      d=gpurun_out/$t/bpmc/inplace_$tag
      timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $d -o run -- \
        python3 tools/bench_build.py --modes inplace --reps 2 --rot 1 > $d.log 2>&1
      rc=$?
      echo "build pmc $tag rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done ;;
  header_probe)
    # the header-only access pattern with each load cache policy: timing,
    # then the L2's memory-side request counters per policy
    tools/gpu_run.sh $t/header_probe 400 python -u tools/header_probe.py || exit $?
    mkdir -p gpurun_out/$t/hpmc
    for m in 0 1 2 3 4; do
      d=gpurun_out/$t/hpmc/mode${m}_REQ
      timeout -s KILL 120 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum \
        TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum --output-format csv -d $d -o run -- \
        python3 tools/header_probe.py --layouts packed --modes $m --writes 1 --rounds 1 \
        --reps 1 --per 3 --warm 0 > $d.log 2>&1
      rc=$?
      echo "hpmc mode $m rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done ;;
  line_probe)
    # how many bytes a scattered access fetches: requests per line for one
    # 64-byte half vs both (tools/line_probe.py), plus the TCC counter names
    timeout -s KILL 60 rocprofv3 -L > gpurun_out/$t/counters_list.txt 2>&1 || true
    tools/gpu_run.sh $t/line_probe 300 python -u tools/line_probe.py || exit $?
    mkdir -p gpurun_out/$t/lpmc
    for h in 1 2 3; do
      for pmc in FETCH_SIZE "TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_32B_sum"; do
        tag=$(echo "$pmc" | cut -d' ' -f1)
        d=gpurun_out/$t/lpmc/halves${h}_$tag
        timeout -s KILL 120 rocprofv3 --pmc $pmc --output-format csv -d $d -o run -- \
          python3 tools/line_probe.py --halves $h --per 2 --reps 1 > $d.log 2>&1
        rc=$?
        echo "lpmc halves $h $tag rc=$rc"
        [ $rc -eq 0 ] || exit $rc
      done
    done ;;
  bubble)
    # TCC_BUBBLE (the 128-byte requests in rocprofv3's FETCH_SIZE formula)
    # and the DRAM read requests, for one / both line halves, the
    # header-only kernel and the streaming checksum kernel
    mkdir -p gpurun_out/$t/bpmc
    for leg in h1 h3 iphdr stream; do
      case $leg in
        h1) cmd="python3 tools/line_probe.py --halves 1 --per 2 --reps 1" ;;
        h3) cmd="python3 tools/line_probe.py --halves 3 --per 2 --reps 1" ;;
        iphdr) cmd="python3 tools/iphdr_probe.py --layouts packed --legs inplace --rounds 1 --reps 1 --per 3 --warm 0 --no-ref" ;;
        stream) cmd="python3 bench.py --steps 3 --warmup 1 --no-graph --ramp-ms 0 --reps 1 --no-ceiling --no-calibrate --no-cpu-baseline --no-order-ab" ;;
      esac
      d=gpurun_out/$t/bpmc/${leg}_BUBBLE
      timeout -s KILL 120 rocprofv3 --pmc TCC_BUBBLE_sum TCC_EA0_RDREQ_DRAM_sum \
        TCC_EA0_RDREQ_sum --output-format csv -d $d -o run -- $cmd > $d.log 2>&1
      rc=$?
      echo "bpmc $leg rc=$rc"
      [ $rc -eq 0 ] || exit $rc
    done ;;
  profile)
    bash tools/profile_round.sh $t/profile || exit $? ;;
  tail)
    # the persistent grid's tail: per-wave start/end stamps (the stamps
    # variant, tools/wave_tail.py) on config 2, config 5 and two of its shards
    XCSUM_LIB=$PWD/libxudp_amd/variants/stamps/libxcsum.so tools/gpu_run.sh $t/wave_tail 500 \
      python -u tools/wave_tail.py --work c2 c5 c5s0/8 c5s7/8 || exit $? ;;
  shards)
    # config 5 whole, and shards 0 and 7 of 8 timed alone (bench.py --shard)
    for a in "--config 5" "--config 5 --shard 0/8" "--config 5 --shard 7/8"; do
      n=$(echo "$a" | sed 's/--config 5//; s/ --shard /_shard/; s/\//of/')
      tools/gpu_run.sh "$t/bench_c5$n" 400 \
        python -u bench.py --steps 50 --warmup 5 --no-cpu-baseline $a || exit $?
    done ;;
  sweep5)
    # config 5 geometry x blocks-per-CU sweep on the current kernels (the
    # sweep variant carries the extra geometries, -DXCSUM_SWEEP_GEOMS)
    XCSUM_LIB=$PWD/libxudp_amd/variants/sweep/libxcsum.so tools/gpu_run.sh $t/sweep5 600 \
      python -u tools/sweep.py --config 5 --rounds 3 --launches 10 \
      --geoms "${SWEEP_GEOMS:-64,1,9;64,2,9;64,1,12;64,2,6;32,2,9;64,3,6;32,1,6;16,1,12}" \
      --bpc "${SWEEP_BPC:-1,2,3,4}" --orders="-1,0;4,2;0,0" || exit $? ;;
  claim)
    # the claimed tail (XCSUM_TUNE_CLAIM) against the static schedule: config
    # 5 whole and one shard, config 2; then the wave stamps with a claim setting
    C="${CLAIMS:-64,0;60,16;56,16;56,4;48,16;48,64;32,16}"
    tools/gpu_run.sh $t/claim_c5 600 python -u tools/sweep.py --config 5 --rounds 3 \
      --launches 10 --geoms auto --claims "$C" || exit $?
    tools/gpu_run.sh $t/claim_c5s7 400 python -u tools/sweep.py --config 5 --shard 7/8 \
      --rounds 3 --launches 20 --geoms auto --claims "$C" || exit $?
    tools/gpu_run.sh $t/claim_c2 400 python -u tools/sweep.py --config 2 --rounds 3 \
      --launches 50 --geoms auto --claims "$C" || exit $?
    XCSUM_LIB=$PWD/libxudp_amd/variants/stamps/libxcsum.so tools/gpu_run.sh $t/wave_tail_claim \
      500 python -u tools/wave_tail.py --work c2 c5 c5s7/8 --claim "${TAIL_CLAIM:-56,16}" \
      || exit $? ;;
  claimtest)
    # the claimed-tail A/B kernels live in the variant builds only
    XCSUM_LIB=$PWD/libxudp_amd/variants/sweep/libxcsum.so tools/gpu_run.sh $t/pytest_claim 600 \
      $P tests/test_gpu_claim.py || exit $? ;;
  scan)
    # config 5 strong scaling projected from every shard of N = 1, 2, 4, 8
    # timed alone on this GPU (tools/shard_scan.py)
    tools/gpu_run.sh $t/shard_scan 600 python -u tools/shard_scan.py || exit $? ;;
  sqtail)
    # the tail in counters: waves, their summed lifetimes
    # (SQ_WAVE_CYCLES, quad-cycles) and the GPU's busy cycles, one pass per
    # workload; tools/sq_summary.py summarises
    mkdir -p gpurun_out/$t/sq
    for w in "c2:--config 2" "c5:--config 5" "c5s7:--config 5 --shard 7/8"; do
      n=${w%%:*}; a=${w#*:}
      d=gpurun_out/$t/sq/$n
      timeout -s KILL 180 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE \
        --output-format csv -d $d -o run -- python3 bench.py $a --steps 3 --warmup 1 --no-graph \
        --ramp-ms 0 --reps 1 --no-ceiling --no-calibrate --no-cpu-baseline --no-order-ab \
        > $d.log 2>&1
      rc=$?
      echo "sq $n rc=$rc"
      [ $rc -eq 0 ] || exit $rc
      python3 tools/sq_summary.py $d > $d.json
    done ;;
  slots)
    # xudp's 4096-byte slots with the like-for-like span probe
    tools/gpu_run.sh $t/bench_c2u 300 python -u bench.py --steps 100 --warmup 5 \
      --no-cpu-baseline --layout umem || exit $? ;;
  host_ab)
    # host batches: this library against round 5's (libxudp_amd/variants/r05,
    # built from git), wide and one-CPU affinity (the staging budget)
    cpu0=$(python3 -c "import os; print(min(os.sched_getaffinity(0)))")
    for lib in new r05; do
      L=$PWD/libxudp_amd/libxcsum.so
      [ $lib = r05 ] && L=$PWD/libxudp_amd/variants/r05/libxcsum.so
      for a in "--config 2 --layout umem" "--config 3 --layout umem" "--config 2 --iphdr-only"; do
        n=$(echo $a | sed 's/--config /c/; s/ --layout umem/u/; s/ --iphdr-only/_iphdr/')
        XCSUM_LIB=$L tools/gpu_run.sh $t/host_${lib}_$n 300 python -u tools/bench_e2e.py $a \
          --reps 5 || exit $?
        XCSUM_LIB=$L tools/gpu_run.sh $t/host_${lib}_${n}_cpu1 300 taskset -c $cpu0 \
          python -u tools/bench_e2e.py $a --reps 5 || exit $?
      done
    done ;;
  *)
    echo "unknown recipe $r"; exit 2 ;;
  esac
done
