#!/bin/bash
# One gpurun job: each GPU step under its own timeout; stop at the first crash / fault / timeout.
# usage: scripts/gpu_job.sh <tag> [steps...]   steps: smoke tests bench benchsmall prof pmc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=${1:-run}; shift
OUT=gpurun_out/$TAG
mkdir -p "$OUT"
export PYTHONUNBUFFERED=1
export TMPDIR=/tmp
run() {  # name timeout cmd...
    local name=$1 to=$2; shift 2
    echo "== $name: $*" | tee -a "$OUT/steps.log"
    timeout -k 10 "$to" "$@" > "$OUT/$name.log" 2>&1
    local rc=$?
    echo "== $name rc=$rc" | tee -a "$OUT/steps.log"
    tail -5 "$OUT/$name.log"
    if [ $rc -ne 0 ]; then
        echo "fatal rc=$rc in $name: stopping" | tee -a "$OUT/steps.log"; exit $rc
    fi
    return 0
}
for s in "$@"; do
    case $s in
        smoke) run smoke 180 python3 -c "import __graft_entry__ as g; g.smoke()" ;;
        tests) run tests 900 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        testsall) run testsall 900 python3 -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread -p no:cacheprovider ;;
        benchsmall) run benchsmall 300 python3 bench.py --events 10000000 --steps 3 --warmup 1 --no-cpu ;;
        bench) run bench 600 python3 bench.py ;;
        prof) run prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/prof" -o run --output-format csv -- python3 bench.py --steps 5 --warmup 2 --no-cpu ;;
        pmc) i=0; for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_INSTS_BRANCH SQ_LDS_BANK_CONFLICT SQ_INSTS_FLAT SQ_INSTS_SMEM" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do i=$((i+1)); run pmc$i 120 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu; done ;;
        c3) run c3 600 python3 scripts/bench_configs.py --only c1,c3m,c4 --c3-steps 2 ;;
        c3prof) run c3prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/c3prof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3m --c3-steps 1 --warmup 1 ;;
        newtests) run newtests 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "regime or long_keys or auto_flush or consumes or many_keys or synthetic" ;;
        dq) run dqtests 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && run dqcfg 300 python3 scripts/bench_configs.py --only c1,c2radix ;;
        c4) run c4 600 python3 scripts/bench_configs.py --only c4 ;;
        c3pmc) i=0; for c in "FETCH_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_INST_CYCLES_VMEM_RD SQ_WAIT_INST_LDS" "TCC_HIT_sum TCC_MISS_sum TCP_TCC_READ_REQ_sum TCP_TCC_WRITE_REQ_sum"; do i=$((i+1)); run c3pmc$i 180 rocprofv3 --pmc $c --kernel-trace -d "$OUT/c3pmc$i" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3m --c3-steps 1 --warmup 0; done ;;
        c3ns) for ns in 8 16 32 64; do run c3ns$ns 300 python3 scripts/bench_configs.py --only c3m --c3-steps 1 --warmup 1 --max-partials $ns; done ;;
        abdq) run abnew 300 python3 bench.py --steps 5 --warmup 2 --no-cpu && run abold 300 env SDG_FU_OLDDQ=1 python3 bench.py --steps 5 --warmup 2 --no-cpu ;;
        phases) for sk in 4 8 16 2 0; do run ph$sk 200 env SDG_FU_SKIP=$sk python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-gather --e2e-steps 0; done; for sk in 2 0; do run phold$sk 200 env SDG_FU_OLDDQ=1 SDG_FU_SKIP=$sk python3 bench.py --steps 3 --warmup 1 --no-cpu --no-parity --no-gather --e2e-steps 0; done; grep -o '"ms_chain_match": [0-9.]*' $OUT/ph*.log ;;
        cpubase) run cpubase 900 python3 scripts/cpu_baselines.py --threads 16 ;;
        c4prof) run c4prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/c4prof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c4 ;;
        c4test) run c4test 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k c4 ;;
        r3tests) run r3tests 900 python3 -u -m pytest tests/test_gpu_robust.py tests/test_gpu_c5.py -m gpu -x -v --timeout 600 --timeout-method thread -p no:cacheprovider ;;
        c5shard) run c5shard 900 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 ;;
        c5prof) run c5prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/c5prof" -o run --output-format csv -- python3 bench.py --config c5 --c5-shard 0/8 --steps 1 --warmup 1 --no-parity --no-gather ;;
        cfgs) run cfgs 900 python3 scripts/bench_configs.py --only c3m,c3md,c2generic,c4 --c3-steps 2 ;;
        cfgshbm) run cfgshbm 900 env SDG_NFA_HBM=1 python3 scripts/bench_configs.py --only c3md,c2generic --c3-steps 2 ;;
        c5host) run c5host 900 env SDG_HOST_PROF=1 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-parity --no-gather ;;
        kt) run kt 900 python3 -u -m pytest tests/test_gpu_keytab.py tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "keytab or keys or regime or c3 or c4" ;;
        cfgs3) run cfgs3 900 python3 scripts/bench_configs.py --only c3m,c3md,c2generic --c3-steps 2 ;;
        purge) run purge 900 python3 -u -m pytest tests/test_gpu_select.py tests/test_gpu_parity.py tests/test_gpu_snapshot.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "purge or Purge or absent or Absent or select or snapshot" ;;
        c3mdprof) run c3mdprof 600 rocprofv3 --kernel-trace --stats -d "$OUT/c3mdprof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 1 ;;
        churn) run churn 600 python3 -u -m pytest tests/test_gpu_churn.py -m gpu -x -v -s --timeout 500 --timeout-method thread -p no:cacheprovider ;;
        ldssweep) for b in 36864 18432 12288 9216 6144 3072; do run lds$b 300 env SDG_NFA_LDS=$b python3 scripts/bench_configs.py --only c3md,c2generic --c3-steps 1 --warmup 1; done; grep -h "^{" $OUT/lds*.log ;;
        mixed) run mixed 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_select.py tests/test_gpu_snapshot.py tests/test_gpu_robust.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c4 or absent or Absent or snapshot or select or failed or corrupt or mixed" ;;
        c4b) run c4b 600 python3 scripts/bench_configs.py --only c4 && run c4bhost 600 env SDG_NO_DEVMIX=1 python3 scripts/bench_configs.py --only c4 ;;
        c5lane) run c5a 600 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-parity --no-gather && run c5b 600 env SDG_CARRY_LANE=1 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-parity --no-gather; grep -h "^{" $OUT/c5a.log $OUT/c5b.log | python3 -c "import json,sys; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_ms']) for l in sys.stdin]" ;;
        pmc2) i=0; for c in "FETCH_SIZE" "WRITE_SIZE"; do i=$((i+1)); run pmc$i 180 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-parity --no-gather --e2e-steps 0; done ;;
        c3pmc2) i=0; for c in "FETCH_SIZE" "WRITE_SIZE" "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS"; do i=$((i+1)); run c3pmc$i 180 rocprofv3 --pmc $c --kernel-trace -d "$OUT/c3pmc$i" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 0; done ;;
        ldsconf) run ldsconf 180 rocprofv3 --pmc SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_BUSY_CYCLES SQ_WAVE_CYCLES --kernel-trace -d "$OUT/ldsconf" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 0 ;;
        c5) run c5 600 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-gather ;;
        seq3) run seq3 900 python3 -u -m pytest tests/test_gpu_seq3.py tests/test_gpu_snapshot.py tests/test_gpu_robust.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && run seq3p 900 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "c3 or many_keys" ;;
        seq3cfg) run seq3cfg 600 python3 scripts/bench_configs.py --only c3md,c3m --c3-steps 3 && run seq3gen 600 env SDG_NO_SEQ3=1 python3 scripts/bench_configs.py --only c3md --c3-steps 2 ;;
        seq3prof) run seq3prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/seq3prof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 2 --warmup 1 ;;
        s3ab) run s3g16 600 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3g8 600 env SDG_S3_G=8 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3pmc 180 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d "$OUT/s3pmc" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 0 && run s3pmcw 180 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/s3pmcw" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 0 ;;
        mr) run mr 600 python3 -u -m pytest tests/test_gpu_multirank.py -m gpu -x -v --timeout 500 --timeout-method thread -p no:cacheprovider ;;
        s3ab2) run s3f16 600 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3f8 600 env SDG_S3_G=8 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3gen 600 env SDG_S3_GENERIC=1 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3prof 600 rocprofv3 --kernel-trace --stats -d "$OUT/s3prof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 2 --warmup 1 ;;
        s3pmc2) run s3sw 600 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3sw8 600 env SDG_S3_G=8 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && i=0 && for c in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES SQ_BUSY_CYCLES" "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_FLAT SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS" "TCP_TCC_READ_REQ_sum TCC_HIT_sum TCC_MISS_sum" "FETCH_SIZE"; do i=$((i+1)); run s3c$i 180 rocprofv3 --pmc $c --kernel-trace -d "$OUT/s3c$i" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 1 --warmup 1 || break; done ;;
        cfgall) run cfgall 900 python3 scripts/bench_configs.py --only c1,c3m,c3md,c4 --c3-steps 3 ;;
        s3sel) run s3t 600 python3 -u -m pytest tests/test_gpu_seq3.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && run s3tb 600 env SDG_S3_BRANCH=1 python3 -u -m pytest tests/test_gpu_seq3.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider -k "shapes or within" && run s3sel 600 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3br 600 env SDG_S3_BRANCH=1 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run s3sel16 600 env SDG_S3_G=16 python3 scripts/bench_configs.py --only c3md --c3-steps 3 ;;
        mrbench) run mrbench 600 env SDG_BENCH_BACKEND=gloo SDG_BENCH_SHARE_GPU=1 python3 -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --steps 3 --warmup 1 --events 30000000 --no-cpu ;;
        wps) for r in 1 2; do run w8_$r 300 env SDG_FU_WPS=8 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-gather --e2e-steps 0 && run w6_$r 300 env SDG_FU_WPS=6 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-gather --e2e-steps 0; done; grep -h "^{" $OUT/w*.log | python3 -c "import json,sys; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_ms']['ms_chain_match']) for l in sys.stdin]" ;;
        cskip) run cskt 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robust.py tests/test_fallbacks.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && for r in 1 2; do run ck_$r 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-gather --e2e-steps 0 && run nk_$r 300 env SDG_FU_NOSKIP=1 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-gather --e2e-steps 0; done; grep -h "^{" $OUT/ck_*.log $OUT/nk_*.log | python3 -c "import json,sys; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_ms']['ms_chain_match'], json.loads(l).get('parity',{}).get('bit_exact')) for l in sys.stdin]" ;;
        rxab) run rxt 900 env SDG_RX_TILE=16384 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_seq3.py tests/test_fallbacks.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && for r in 1 2; do run rb_$r 300 env SDG_RX_TILE=16384 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-gather --e2e-steps 0 && run rs_$r 300 env SDG_RX_TILE=8192 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-gather --e2e-steps 0; done && grep -h "^{" $OUT/rb_*.log $OUT/rs_*.log | python3 -c "import json,sys; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_ms']['ms_kg_scatter'], json.loads(l)['roofline']['kernel_ms']['ms_chain_match'], json.loads(l).get('parity',{}).get('bit_exact')) for l in sys.stdin]" && run rc5b 600 env SDG_RX_TILE=16384 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-gather && run rc5s 600 env SDG_RX_TILE=8192 python3 bench.py --config c5 --c5-shard 0/8 --steps 3 --warmup 1 --no-gather && run rxw 180 env SDG_RX_TILE=16384 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d "$OUT/rxw" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-parity --no-gather --e2e-steps 0 ;;
        c4hp) run c4hp 600 env SDG_HOST_PROF=1 python3 scripts/bench_configs.py --only c4 ;;
        c4ab) run c4t 600 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_select.py -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider -k "c4 or absent or collision" && run c4new 600 python3 scripts/bench_configs.py --only c4 && run c4hp 600 env SDG_HOST_PROF=1 python3 scripts/bench_configs.py --only c4 && run c4exact 600 env SDG_SCHED_EXACT=1 python3 scripts/bench_configs.py --only c4 ;;
        c3rx) for r in 1 2; do run c3b_$r 300 env SDG_RX_TILE=16384 python3 scripts/bench_configs.py --only c3md --c3-steps 3 && run c3s_$r 300 env SDG_RX_TILE=8192 python3 scripts/bench_configs.py --only c3md --c3-steps 3; done && run c3rxprof 300 rocprofv3 --kernel-trace --stats -d "$OUT/c3rxprof" -o run --output-format csv -- python3 scripts/bench_configs.py --only c3md --c3-steps 2 --warmup 1 && grep -h "^{" $OUT/c3b_*.log $OUT/c3s_*.log ;;
        emab) run emt 900 python3 -u -m pytest tests/test_gpu_parity.py tests/test_gpu_robust.py -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider && for r in 1 2; do run e8_$r 300 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-gather --e2e-steps 0 && run e6_$r 300 env SDG_FU_WPS=6 python3 bench.py --steps 10 --warmup 2 --no-cpu --no-parity --no-gather --e2e-steps 0; done && grep -h "^{" $OUT/e8_*.log $OUT/e6_*.log | python3 -c "import json,sys; [print(json.loads(l)['ms_per_step'], json.loads(l)['roofline']['kernel_ms']['ms_kg_scatter'], json.loads(l)['roofline']['kernel_ms']['ms_chain_match'], json.loads(l).get('parity',{}).get('bit_exact')) for l in sys.stdin]" && i=0 && for c in "FETCH_SIZE" "WRITE_SIZE"; do i=$((i+1)); run pmc$i 180 rocprofv3 --pmc $c --kernel-trace -d "$OUT/pmc$i" -o run --output-format csv -- python3 bench.py --steps 2 --warmup 1 --no-cpu --no-parity --no-gather --e2e-steps 0; done ;;
        *) echo "unknown step $s" ;;
    esac
done
echo "job done"
