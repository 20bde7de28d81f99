#!/bin/bash
# One GPU session on the MI355X box: parity tests, smoke, bench, rocprofv3 kernel stats.
# Each GPU step has its own time limit; a fault / abort / segfault / timeout ends the session.
# Usage: tools/gpu_session.sh [steps...]   steps: tests smoke bench prof pmc (default: all)
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
STEPS=${*:-"tests smoke bench prof"}
TAG=${TAG:-r01}

run() {  # name seconds cmd...
    local name=$1 t=$2
    shift 2
    echo "=== $name (limit ${t}s): $*"
    local t0=$(date +%s)
    timeout -k 10 "$t" "$@" > "gpurun_out/$name.log" 2>&1
    local rc=$?
    echo "=== $name rc=$rc ($(( $(date +%s) - t0 ))s)"
    tail -n 25 "gpurun_out/$name.log"
    return $rc
}
fatal() {  # exit codes after which nothing more may touch the GPU
    case $1 in 0|1|2|3|4|5) return 1 ;; *) return 0 ;; esac
}

[ -f maximumareacoverageoptimization.jl_amd/libmaxcover.so ] || make -s -C maximumareacoverageoptimization.jl_amd/csrc
[ -f oracle/libref_cpu.so ] || make -s -C oracle

for s in $STEPS; do
    case $s in
    tests)
        run pytest_gpu 600 python -u -m pytest tests -m gpu -x -v -rfE -p no:cacheprovider --timeout 120 --timeout-method thread ; rc=$? ;;
    testsall)   # every GPU test, no stop at the first failure
        run pytest_gpu_all 900 python -u -m pytest tests -m gpu -v -rfE -p no:cacheprovider --timeout 120 --timeout-method thread ; rc=$?
        [ $rc -eq 1 ] && rc=0 ;;
    fused)   # the fused chain's tests alone
        run pytest_fused 400 python -u -m pytest tests/test_gpu_fused.py -x -v -rfE -p no:cacheprovider --timeout 120 --timeout-method thread ; rc=$? ;;
    mads)   # the native MADS loop's tests alone
        run pytest_mads 400 python -u -m pytest tests -m gpu -k "mads" -x -v -rfE -p no:cacheprovider --timeout 120 --timeout-method thread ; rc=$? ;;
    gather)   # RCCL world-1 exchange costs (dist.PollGather / DeviceGather)
        run gather 200 python tools/time_gather.py ; rc=$? ;;
    smoke)
        run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ; rc=$? ;;
    benchq)
        run benchq 300 python bench.py --no-cpu ; rc=$? ;;
    benchplain)   # config 4, polls launched one after another (no doorbell)
        run benchplain 300 python bench.py --no-cpu --step-mode plain ; rc=$? ;;
    bench)
        run bench 400 python bench.py ; rc=$?
        grep '^{' gpurun_out/bench.log > gpurun_out/bench_${TAG}.json ;;
    algos)
        for a in tiled poll auto; do
            run bench_$a 600 python bench.py --no-cpu --algo $a --steps 30 ; rc=$?
            fatal $rc && break
        done ;;
    diag)
        make -s -C maximumareacoverageoptimization.jl_amd/csrc diag
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diag 600 python tools/diag_poll.py ; rc=$? ;;
    diag5)
        make -s -C maximumareacoverageoptimization.jl_amd/csrc diag
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diag5 600 python tools/diag_poll.py --config 5 ; rc=$? ;;
    diagfiw)
        make -s -C maximumareacoverageoptimization.jl_amd/csrc diag
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diagfiw 300 python tools/diag_fiw.py ; rc=$? ;;
    diagidx)
        make -s -C maximumareacoverageoptimization.jl_amd/csrc diag
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diagidx 600 python tools/diag_index.py ; rc=$? ;;
    weak2)   # rehearsal of the N=2 path on one GPU (gloo; both ranks on device 0)
        MAXCOVER_BENCH_DEVICE=0 run weak2 300 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 \
            --no-cpu --dist-backend gloo --steps 20 ; rc=$? ;;
    self2)   # bench.py --gpus 2 with no external launcher: it starts its two ranks itself (gloo; both on device 0)
        MAXCOVER_BENCH_DEVICE=0 run self2 300 python bench.py --gpus 2 --no-cpu --dist-backend gloo --steps 20 ; rc=$?
        grep '^{' gpurun_out/self2.log > gpurun_out/self2_${TAG}.json ;;
    diagor)   # phase times of the union pass on the config-5 regression poll at ell 5 / 4 / 3
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diagor 300 python tools/diag_or.py ; rc=$? ;;
    probeka)  # can a launch carry the 12-KB closure candidate as kernel arguments? (tools/probe)
        [ -x tools/probe/kernarg_probe ] || /opt/rocm/bin/hipcc --offload-arch=gfx950 -O2 tools/probe/kernarg_probe.hip -o tools/probe/kernarg_probe
        run probeka 60 tools/probe/kernarg_probe ; rc=$? ;;
    c5walks)  # the config-5 regression poll at ell 5..1 through each walk (per-kernel times)
        run c5walks 300 python tools/c5_walks.py ; rc=$? ;;
    c5polls)  # per-poll kernel times of the config-5 loop; the slowest polls saved for analysis
        run c5polls 600 python tools/c5_polls.py ; rc=$? ;;
    c5x2)    # rehearsal of the N=2 config-5 path (sharded MADS) on one GPU (gloo; both ranks on device 0)
        MAXCOVER_BENCH_DEVICE=0 run c5x2 400 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29534 bench.py --gpus 2 \
            --config 5 --no-cpu --dist-backend gloo --steps 2 --warmup 1 --mads-mode shard ; rc=$?
        grep '^{' gpurun_out/c5x2.log > gpurun_out/c5x2_${TAG}.json ;;
    c5x2s)   # the speculative N=2 config-5 loop on one GPU (gloo; both ranks on device 0)
        MAXCOVER_BENCH_DEVICE=0 run c5x2s 400 python -m torch.distributed.run --nnodes=1 \
            --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29535 bench.py --gpus 2 \
            --config 5 --no-cpu --dist-backend gloo --steps 2 --warmup 1 --mads-mode speculate ; rc=$?
        grep '^{' gpurun_out/c5x2s.log > gpurun_out/c5x2s_${TAG}.json ;;
    probe)
        { nproc; python3 -c "import os; print(os.cpu_count(), len(os.sched_getaffinity(0)))";
          cat /sys/fs/cgroup/cpu.max 2>/dev/null; lscpu | grep -E 'Model name|Socket|Core|Thread'; 
          echo OMP=$OMP_NUM_THREADS; } > gpurun_out/probe.log 2>&1; cat gpurun_out/probe.log; rc=0 ;;
    benchc)
        run benchc 400 python bench.py --disks clustered --no-cpu ; rc=$?
        grep '^{' gpurun_out/benchc.log > gpurun_out/benchc_${TAG}.json ;;
    bench3)
        run bench3 600 python bench.py --config 3 --no-cpu ; rc=$? ;;
    chains5)   # config 5 through each forced chain
        for c in five fused; do
            run bench5_$c 600 python bench.py --config 5 --steps 2 --warmup 1 --no-cpu --chain $c ; rc=$?
            fatal $rc && break
        done ;;
    chains4)   # config 4 through each forced chain
        for c in five fused; do
            run bench4_$c 300 python bench.py --no-cpu --no-extras --chain $c ; rc=$?
            fatal $rc && break
        done ;;
    bench5)
        run bench5 600 python bench.py --config 5 --steps 3 --warmup 1 --no-cpu ; rc=$? ;;
    shards)   # per-rank chain floor of the strong split: rank 0's shard alone on one GPU
        for P in 2 4 8; do
            run shard$P 300 python bench.py --no-cpu --shard-of $P ; rc=$?
            fatal $rc && break
        done ;;
    dshards)   # per-rank floor of a disk split: rank 0's disks alone on one GPU
        for P in 2 4 8; do
            run dshard$P 300 python bench.py --no-cpu --no-extras --disk-shard-of $P ; rc=$?
            fatal $rc && break
        done ;;
    prof5)    # kernel stats of the config-5 MPC loop and of the clustered config-4 poll
        rm -rf gpurun_out/prof5 gpurun_out/profc
        run prof5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof5 -o run \
            -- python3 bench.py --config 5 --steps 2 --warmup 1 --no-cpu ; rc=$?
        fatal $rc || run profc 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/profc -o run \
            -- python3 bench.py --disks clustered --steps 10 --warmup 2 --no-cpu --no-extras ; rc=$? ;;
    cprof)   # the single-candidate closure path: latency + kernel stats
        rm -rf gpurun_out/cprof
        run cprof 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/cprof -o run \
            -- python3 tools/closure_prof.py ; rc=$? ;;
    bench2)
        run bench2 600 python bench.py --config 2 --no-cpu ; rc=$? ;;
    prof)
        rm -rf gpurun_out/prof
        run prof 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof -o run \
            -- python3 bench.py --steps 10 --warmup 2 --no-cpu --no-extras ; rc=$?
        find gpurun_out/prof -name '*stats*' | head ;;
    pmc)
        rm -rf gpurun_out/pmc_fetch gpurun_out/pmc_write
        run pmc_fetch 900 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run \
            -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras ; rc=$?
        if ! fatal $rc; then
            run pmc_write 900 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run \
                -- python3 bench.py --steps 5 --warmup 1 --no-cpu --no-extras ; rc=$?
        fi
        fatal $rc || python3 tools/pmc_traffic.py gpurun_out/pmc_fetch gpurun_out/pmc_write --config 4 \
            --chain 'mac::prep_x_kernel<false>;mac::fiw_kernel<true>;mac::fin2_kernel<true>' \
            --out gpurun_out/pmc_traffic_config4.json ;;
    diagprep)   # prep launch: per-workgroup spans; phases of the first 64 (diagnostic build)
        MAXCOVER_LIB=$PWD/maximumareacoverageoptimization.jl_amd/libmaxcover_diag.so \
            run diagprep 300 python tools/diag_prep.py ; rc=$? ;;
    pmccp)   # the fresh PMC file where bench.py looks for it (attached while src_sha matches)
        cp gpurun_out/pmc_traffic_config4.json profiles/pmc_traffic_config4.json ; rc=$? ;;
    *) echo "unknown step $s"; rc=0 ;;
    esac
    if fatal $rc; then echo "=== stopping: $s exited $rc"; exit $rc; fi
done
echo "=== session done"
