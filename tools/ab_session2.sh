#!/bin/bash
# The GPU calls of round 2's second session, one step per call:
#   gpurun -- bash tools/ab_session2.sh <step>        (logs in gpurun_out/<step>/)
# Results are indexed in profiles/README.md ("Round 2, second session").
# Steps that compare builds need the variant libraries first, e.g.
#   make -C libxudp_amd variant NAME=ntrec DEFS=-DXCSUM_RX_NTREC=1
# (the knobs each step compared are named in profiles/README.md).
set -e
export TMPDIR=/tmp
case "$1" in
s3)

  tools/gpu_run.sh s3/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s3/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tools/gpu_run.sh s3/bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
  tools/gpu_run.sh s3/slot_small 200 python tools/slot_probe.py --small
  for c in 4 5; do
    tools/gpu_run.sh s3/fetch$c 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s3/fetch$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
    tools/gpu_run.sh s3/write$c 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/s3/write$c -o run -- python3 bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
  done
  tools/gpu_run.sh s3/sweep5_bpc 300 python tools/sweep.py --config 5 --geoms "64,1,9" --bpc 1,2,3,4 --orders=-1,0 --rounds 3 --launches 10
  ;;
s4)
  # round-2 session-2 A/B call: config 5 first-row temporal loads / all temporal,
  # receive kernel capped at 3 waves/SIMD, config 3 in xudp's slot layout sweep
  mkdir -p gpurun_out/s4
  for r in 1 2; do
    for v in cur edget nt0; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      XCSUM_LIB=$L tools/gpu_run.sh s4/c5_${v}_$r 200 python bench.py --config 5 --steps 10 --warmup 2 --reps 3 --no-cpu-baseline --no-ceiling
    done
  done
  for v in edget nt0; do
    XCSUM_LIB=libxudp_amd/variants/$v/libxcsum.so tools/gpu_run.sh s4/fetch5_$v 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/s4/fetch5_$v -o run -- python3 bench.py --config 5 --steps 10 --warmup 2 --no-cpu-baseline --no-graph --ramp-ms 0 --reps 1 --no-ceiling
  done
  ROUNDS=2 tools/ab_rx_libs.sh gpurun_out/s4/rx 2,4 auto rxw3
  tools/gpu_run.sh s4/sweep3_umem 300 python tools/sweep.py --config 3 --layout umem --geoms "4,1,2;8,1,2;4,2,2;2,1,4" --bpc 0,2,4,8 --orders="-1,0;0,0;3,4;7,4" --rounds 3 --launches 20
  ;;
s5)
  # A/B: sparse fallback of the stream kernel at G = 8 (config 3 in xudp's
  # slots), nontemporal receive-record stores
  mkdir -p gpurun_out/s5
  for r in 1 2; do
    for v in cur sg8; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      XCSUM_LIB=$L tools/gpu_run.sh s5/c3u_${v}_$r 200 python bench.py --config 3 --layout umem --steps 100 --warmup 5 --reps 3 --no-cpu-baseline --no-ceiling
      XCSUM_LIB=$L tools/gpu_run.sh s5/c3p_${v}_$r 200 python bench.py --config 3 --steps 100 --warmup 5 --reps 3 --no-cpu-baseline --no-ceiling
    done
  done
  ROUNDS=2 tools/ab_rx_libs.sh gpurun_out/s5/rx 2,4,5 auto ntrec
  ;;
s6)
  # full GPU suite on nontemporal receive records; A/B nontemporal result /
  # in-place stores in the checksum kernels (flags none / INPLACE / INPLACE+IPHDR)
  mkdir -p gpurun_out/s6
  tools/gpu_run.sh s6/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s6/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
  for r in 1 2; do
    for v in cur ntst; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      for fl in none inplace inplace,iphdr verify; do
        XCSUM_LIB=$L tools/gpu_run.sh s6/c2_${v}_${fl/,/_}_$r 200 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags $fl --rounds 3 --launches 20
      done
      XCSUM_LIB=$L tools/gpu_run.sh s6/c2u_${v}_inplace_iphdr_$r 200 python tools/sweep.py --config 2 --layout umem --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags inplace,iphdr --rounds 3 --launches 20
      XCSUM_LIB=$L tools/gpu_run.sh s6/c3_${v}_$r 200 python tools/sweep.py --config 3 --geoms 64,0,8 --bpc 0 --orders=-1,0 --rounds 3 --launches 40
      XCSUM_LIB=$L tools/gpu_run.sh s6/c5_${v}_$r 200 python tools/sweep.py --config 5 --geoms 64,1,9 --bpc 0 --orders=-1,0 --rounds 2 --launches 10
    done
  done
  ;;
s7)
  # copy-free small-batch host path (XCSUM_DIRECT_MAX) vs current: correctness
  # (TX ring harness, host-path GPU tests) and per-call cost by batch size
  mkdir -p gpurun_out/s7
  V=libxudp_amd/variants/direct
  LD_LIBRARY_PATH=$V tools/gpu_run.sh s7/ring_direct_check 200 tests/c/umem_ring
  XCSUM_LIB=$V/libxcsum.so tools/gpu_run.sh s7/pytest_host_direct 300 python -u -m pytest tests/test_gpu_host_path.py tests/test_gpu_config1.py tests/test_gpu_fuzz.py -m gpu -x -q --timeout 120 --timeout-method thread
  for r in 1 2; do
    tools/gpu_run.sh s7/ring_cur_$r 300 tests/c/umem_ring --bench 1,16,100,1024,4096
    LD_LIBRARY_PATH=$V tools/gpu_run.sh s7/ring_direct_$r 300 tests/c/umem_ring --bench 1,16,100,1024,4096
  done
  ;;
s8)
  # host path per-call cost: copy-free small batches, and spin-wait on the slot event
  mkdir -p gpurun_out/s8
  for r in 1 2 3; do
    for v in cur direct dspin; do
      L=; [ $v = cur ] || L=libxudp_amd/variants/$v
      LD_LIBRARY_PATH=$L tools/gpu_run.sh s8/ring_${v}_$r 300 tests/c/umem_ring --bench 1,16,100,1024
    done
  done
  ;;
s10)
  # full GPU suite + TX ring harness + end-to-end bench on the final host path
  mkdir -p gpurun_out/s10
  tools/gpu_run.sh s10/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s10/ring_check 200 tests/c/umem_ring
  tools/gpu_run.sh s10/ring_bench 300 tests/c/umem_ring --bench 1,16,100,1024,4096
  tools/gpu_run.sh s10/e2e 300 python tools/bench_e2e.py
  ;;
s11)
  # stream receive kernel (64,8,3) for packed small frames: receive tests, then
  # every receive mode on config 3 against the group / wide kernels
  tools/gpu_run.sh s11/pytest_rx 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_offsets.py -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s11/bench_rx3 300 python tools/bench_rx.py --configs 3 --geoms "auto;4,2,1;4,2,0;64,8,3"
  tools/gpu_run.sh s11/bench_rx3_umem 300 python tools/bench_rx.py --configs 3 --layout umem --geoms "auto;64,8,3"
  ;;
s12)
  # the stream receive kernel as the small-frame default (plain and VERIFY;
  # sparse batches fall back to (4,2,0) / (4,2,1)): whole suite, every mode
  tools/gpu_run.sh s12/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s12/bench_rx 300 python tools/bench_rx.py --configs 2,4,3,5
  tools/gpu_run.sh s12/bench_rx3_umem 300 python tools/bench_rx.py --configs 3 --layout umem --geoms "auto;4,2,0;4,2,1"
  tools/gpu_run.sh s12/e2e 300 python tools/bench_e2e.py
  ;;
s13)
  # receive host path: sparse batches in a pageable UMEM gathered frame by
  # frame (XCSUM_RX_GATHER) vs the range copy, MTU and 64-byte frames
  tools/gpu_run.sh s13/pytest_rx 600 python -u -m pytest tests/test_gpu_rx.py -m gpu -x -q --timeout 120 --timeout-method thread
  for v in cur nogather; do
    L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
    for c in 2 3; do
      XCSUM_LIB=$L tools/gpu_run.sh s13/e2e_umem_c${c}_$v 300 python tools/bench_e2e.py --config $c --layout umem --reps 3
    done
  done
  ;;
s14)
  # gather only where frames fill < 1/8 of the range (and the TX host batch
  # too): host-path and receive tests, e2e on xudp's chunks, MTU and 64 B
  tools/gpu_run.sh s14/pytest 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_host_path.py tests/test_gpu_host_direct.py -m gpu -x -q --timeout 120 --timeout-method thread
  for c in 2 3; do
    tools/gpu_run.sh s14/e2e_umem_c$c 300 python tools/bench_e2e.py --config $c --layout umem --reps 3
  done
  ;;
s15)
  # whole GPU suite, smoke and the driver's bench command on the session's final code
  tools/gpu_run.sh s15/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s15/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tools/gpu_run.sh s15/bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
  tools/gpu_run.sh s15/ring_bench 300 tests/c/umem_ring --bench 1,16,100,1024,4096
  ;;
s16)
  # sparse batches in a registered UMEM read in place without XCSUM_F_ZEROCOPY
  tools/gpu_run.sh s16/pytest 600 python -u -m pytest tests/test_gpu_rx.py tests/test_gpu_host_path.py tests/test_gpu_host_direct.py tests/test_capi.py -m gpu -x -q --timeout 120 --timeout-method thread
  for c in 2 3; do
    tools/gpu_run.sh s16/e2e_umem_c$c 300 python tools/bench_e2e.py --config $c --layout umem --reps 3
  done
  ;;
s17)
  # any sparse batch in a registered UMEM read in place (2x rule): whole
  # suite, TX ring harness by batch size, end to end on xudp's chunks
  tools/gpu_run.sh s17/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s17/ring_bench 300 tests/c/umem_ring --bench 1,16,100,1024,4096
  for c in 2 3 4; do
    tools/gpu_run.sh s17/e2e_umem_c$c 300 python tools/bench_e2e.py --config $c --layout umem --reps 3
  done
  tools/gpu_run.sh s17/e2e_packed_c2 300 python tools/bench_e2e.py --config 2 --reps 3
  ;;
s18)
  # config 5: visiting orders (2^R regions of 2^T-frame tiles) against the
  # plain cyclic assignment: blocked (one region per wave) to interleaved
  tools/gpu_run.sh s18/sweep5_orders 300 python tools/sweep.py --config 5 --geoms 64,1,9 --bpc 0 --orders="0,0;11,0;10,0;8,0;5,0;11,2;5,2;3,4" --rounds 2 --launches 8
  ;;
s19)
  # config 5 orders, finer; and the MTU configs (2, 4) under the same orders
  tools/gpu_run.sh s19/sweep5_orders 400 python tools/sweep.py --config 5 --geoms 64,1,9 --bpc 0 --orders="0,0;5,2;5,1;5,3;4,2;6,2;7,2;3,2;5,0" --rounds 3 --launches 8
  tools/gpu_run.sh s19/sweep2_orders 300 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders="0,0;5,2;5,4;3,4" --rounds 3 --launches 20
  ;;
s20)
  # packed MTU configs: orders swept finer, then the bench itself (graph
  # replay) with XCSUM_ORDER forced vs automatic, interleaved processes
  tools/gpu_run.sh s20/sweep2_orders 400 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders="0,0;3,4;2,4;3,3;3,5;4,4;2,5;3,6;1,4" --rounds 3 --launches 20
  tools/gpu_run.sh s20/sweep4_orders 300 python tools/sweep.py --config 4 --geoms 16,2,6 --bpc 0 --orders="0,0;3,4;2,4;4,4;3,5" --rounds 3 --launches 20
  for r in 1 2; do
    for o in auto 3,4 2,4; do
      if [ $o = auto ]; then E=; else E="XCSUM_ORDER=$o"; fi
      env $E tools/gpu_run.sh s20/bench_c2_${o/,/_}_$r 200 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
    done
  done
  ;;
s21)
  # dense-batch visiting order per geometry (XCSUM_DENSE_ORDER): suite, then
  # the bench per config and flag sweeps against the descriptor-order build
  tools/gpu_run.sh s21/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  for r in 1 2; do
    for v in cur nodense; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      for c in 2 4 5; do
        XCSUM_LIB=$L tools/gpu_run.sh s21/bench_c${c}_${v}_$r 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
      done
      XCSUM_LIB=$L tools/gpu_run.sh s21/flags_c2_${v}_$r 200 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags inplace,iphdr --rounds 2 --launches 20
      XCSUM_LIB=$L tools/gpu_run.sh s21/verify_c2_${v}_$r 200 python tools/sweep.py --config 2 --geoms 16,2,6 --bpc 0 --orders=-1,0 --flags verify --rounds 2 --launches 20
    done
  done
  ;;
s22)
  # dense order for MTU frames: 8 vs 16 regions of 16-frame tiles, in the bench
  for r in 1 2 3; do
    for o in 3,4 4,4 2,4; do
      for c in 2 4; do
        XCSUM_ORDER=$o tools/gpu_run.sh s22/bench_c${c}_${o/,/_}_$r 200 python bench.py --config $c --steps 20 --warmup 5 --no-cpu-baseline --no-ceiling
      done
    done
  done
  ;;
s23)
  # the receive kernels under dense-batch region orders (XCSUM_RX_DENSE)
  for r in 1 2; do
    for o in none 3,6 4,6 5,6; do
      if [ $o = none ]; then E=; else E="XCSUM_RX_DENSE=$o"; fi
      env $E tools/gpu_run.sh s23/rx_${o/,/_}_$r 300 python tools/bench_rx.py --configs 2,4,5 --only verify,csum_verify
    done
  done
  ;;
s24)
  # final tree: whole suite, smoke, driver bench; dense orders for the
  # mid-size geometries (payloads 150 / 400 / 700 B: (8,1,2), (16,1,2), (16,1,3))
  tools/gpu_run.sh s24/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s24/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tools/gpu_run.sh s24/bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
  for p in 150 400 700; do
    tools/gpu_run.sh s24/sweep_p$p 300 python tools/sweep.py --config 2 --payload $p,$p --geoms auto --bpc 0 --orders="-1,0;3,4;4,4;4,2;5,4" --rounds 3 --launches 20
  done
  ;;
s25)
  # the final tree: whole suite and smoke; the mid-size payloads again under the new default
  tools/gpu_run.sh s25/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s25/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  for p in 400 700; do
    tools/gpu_run.sh s25/sweep_p$p 300 python tools/sweep.py --config 2 --payload $p,$p --geoms auto --bpc 0 --orders="-1,0;0,0" --rounds 3 --launches 20
  done
  ;;
s26)
  # sparse batches (xudp's 4096-byte slots): the region order re-swept with
  # round 2's kernels, MTU IPv4 / IPv6 and the in-place header build flags
  tools/gpu_run.sh s26/sweep2u 300 python tools/sweep.py --config 2 --layout umem --geoms auto --bpc 0 --orders="-1,0;4,4;3,4;6,4;5,3;5,5;4,3;6,3" --rounds 3 --launches 20
  tools/gpu_run.sh s26/sweep4u 300 python tools/sweep.py --config 4 --layout umem --geoms auto --bpc 0 --orders="-1,0;4,4;6,4;5,3;5,5" --rounds 3 --launches 20
  tools/gpu_run.sh s26/sweep2u_ip 300 python tools/sweep.py --config 2 --layout umem --geoms auto --bpc 0 --orders="-1,0;4,4;6,4;5,3;5,5" --flags inplace,iphdr --rounds 3 --launches 20
  ;;
s27)
  # stream kernel (config 3): 64-frame groups visited in region order
  # (XCSUM_STREAM_RLOG / _TLOG variants) vs descriptor order; stream tests
  # under one variant
  XCSUM_LIB=libxudp_amd/variants/so3t2/libxcsum.so tools/gpu_run.sh s27/pytest_stream 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_offsets.py -m gpu -x -q --timeout 120 --timeout-method thread
  for r in 1 2; do
    for v in cur so3t2 so4t0 so5t2; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      XCSUM_LIB=$L tools/gpu_run.sh s27/bench_c3_${v}_$r 200 python bench.py --config 3 --steps 100 --warmup 5 --no-cpu-baseline --no-ceiling
    done
  done
  ;;
s28)
  # stream kernel group orders, second set
  for r in 1 2 3; do
    for v in cur so4t0 so3t0 so4t1 so5t0; do
      L=libxudp_amd/libxcsum.so; [ $v = cur ] || L=libxudp_amd/variants/$v/libxcsum.so
      XCSUM_LIB=$L tools/gpu_run.sh s28/bench_c3_${v}_$r 200 python bench.py --config 3 --steps 100 --warmup 5 --no-cpu-baseline --no-ceiling
    done
  done
  ;;
s29)
  # the final tree (stream kernel group order on): whole suite, smoke, the
  # driver's bench, config 3 bench
  tools/gpu_run.sh s29/pytest_gpu 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread
  tools/gpu_run.sh s29/smoke 200 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')"
  tools/gpu_run.sh s29/bench 300 python bench.py --gpus 1 --steps 20 --warmup 5
  tools/gpu_run.sh s29/bench_c3 200 python bench.py --config 3 --steps 100 --no-cpu-baseline
  ;;
*)
  echo "usage: $0 s3|s4|s5|s6|s7|s8|s10|s11|s12|s13|s14|s15|s16|s17|s18|s19|s20|s21|s22|s23|s24|s25|s26|s27|s28|s29" >&2
  exit 2
  ;;
esac
