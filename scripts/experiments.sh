# Named GPU experiments (round 3 and later), one parameterised runner instead of one-off files.
#   gpurun -- 'bash scripts/experiments.sh <name> [args]'
# Every GPU step runs under its own time limit and the chain stops at the first failure.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
name=$1; shift
O=gpurun_out/exp_$name; mkdir -p $O

case $name in
  lib_ab)         # this tree's library vs a variant build (csrc/build.py --variant V -D ...):
                  # args V [pytest files]: GPU tests of the default library, the 4096^2 x 65536
                  # weight-gradient probe and the real 13-layer launch on both, then three
                  # interleaved whole steps
    v=$1; shift; P=vi_normflows_amd/_native/libvinf_hip_$v.so
    if [ $# -gt 0 ]; then
      timeout -k 10 400 python -u -m pytest "$@" -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
      tail -1 $O/pytest.txt
    fi
    for r in 1 2; do
      for lib in default $v; do
        if [ $lib = default ]; then L=""; else L=$P; fi
        VINF_NATIVE_LIB=$L timeout -k 10 200 python -m vi_normflows_amd.bench.wgrad_bench --tag $lib --probe --cases tn4w_real,tn4w_cached --iters 5 >> $O/probe.jsonl || exit 1
        VINF_NATIVE_LIB=$L timeout -k 10 200 python -m vi_normflows_amd.bench.wgrad_bench --tag $lib --layout-probe --layers 13 --iters 3 --layouts 3 >> $O/wg.jsonl || exit 1
      done
    done
    cat $O/probe.jsonl $O/wg.jsonl
    for r in 1 2 3; do
      for lib in default $v; do
        if [ $lib = default ]; then L=""; else L=$P; fi
        VINF_NATIVE_LIB=$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" | tee -a $O/bench.jsonl
      done
    done ;;
  mem_issue)      # per-CU / per-XCD global load & store issue rates (tools/mem_issue_bench.hip)
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/mem_issue_bench.hip -o $O/mem_issue_bench &&
    timeout -k 10 120 $O/mem_issue_bench full > $O/mem.jsonl ;;
  dma)            # LDS-DMA operand stream: segment size x footprint x DMA depth per wave
    /opt/rocm/bin/hipcc -O3 --offload-arch=gfx950 tools/mem_issue_bench.hip -o $O/mem_issue_bench &&
    timeout -k 10 120 $O/mem_issue_bench dma > $O/dma.jsonl ;;
  probe_libs)     # the 4096^2 x 65536 weight-gradient probe on this tree's library and on
                  # variant builds (args: variant names; timing-only probe builds allowed)
    for r in 1 2; do
      for lib in default "$@"; do
        if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
        VINF_NATIVE_LIB=$L timeout -k 10 200 python -m vi_normflows_amd.bench.wgrad_bench --tag $lib --probe --cases tn4w_real,tn4w_cached --iters 5 >> $O/probe.jsonl || exit 1
      done
    done
    cat $O/probe.jsonl ;;
  probe_pmc)      # counter passes of the 4-wave weight-gradient probe (tn4w_real) on this
                  # tree's library and variant builds (args: variant names); pass 1: issue /
                  # FIFO stalls at the SQ, pass 2: TA / TD / TCP stalls
    export TMPDIR=/tmp
    P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_INST_CYCLES_VMEM_RD SQ_ACTIVE_INST_VMEM SQ_VMEM_TA_ADDR_FIFO_FULL SQ_VMEM_TA_CMD_FIFO_FULL SQ_LDS_DATA_FIFO_FULL SQ_LDS_CMD_FIFO_FULL"
    P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES TA_TA_BUSY_sum TA_ADDR_STALLED_BY_TC_CYCLES_sum TD_TD_BUSY_sum TD_TC_STALL_sum TCP_PENDING_STALL_CYCLES_sum TCP_TCR_TCP_STALL_CYCLES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum TCP_UTCL1_SERIALIZATION_STALL_sum"
    P3="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_INST_LEVEL_VMEM SQ_ACTIVE_INST_SCA"
    for lib in default "$@"; do
      if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
      for pp in 1 2 3; do
        eval "C=\$P$pp"
        VINF_NATIVE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${lib}_p$pp -o pmc --output-format csv -- python3 -m vi_normflows_amd.bench.wgrad_bench --probe --cases tn4w_real --iters 3 > $O/${lib}_p$pp.log 2>&1 || { echo P${pp}_FAIL $lib; tail -20 $O/${lib}_p$pp.log; exit 1; }
      done
      python3 -m vi_normflows_amd.bench.pmc_summary $O/${lib}_p1 $O/${lib}_p2 $O/${lib}_p3 > $O/${lib}_summary.txt 2>&1
      echo "== $lib"; grep -A3 tn4w $O/${lib}_summary.txt
    done ;;
  wgrad_probe)    # TN weight-gradient loop: real vs cache-resident operands vs the NT kernel
    timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag ${1:-cur} --probe --iters 5 > $O/probe.jsonl &&
    true ;;
  wgrad_quick)    # weight-gradient correctness + the real deferred launch + the TN/NT probe
    timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 &&
    timeout -k 10 180 python -m vi_normflows_amd.bench.wgrad_bench --tag ${1:-cur} --layers 13 >> $O/wg.jsonl &&
    timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag ${1:-cur} --probe --iters 5 >> $O/probe.jsonl ;;
  wgrad_pmc)      # L2 hit / miss and wave-state counters of the TN / NT probe (one counter pass)
    export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAIT_ANY SQ_WAVE_CYCLES SQ_VALU_MFMA_BUSY_CYCLES SQ_BUSY_CYCLES \
      -d $O/pmc -o probe --output-format csv -- python3 -m vi_normflows_amd.bench.wgrad_bench --probe --iters 2 > $O/probe.log 2>&1 ;;
  step_ab)        # whole-step A/B of an environment switch: args NAME VALUE_A VALUE_B [rounds]
    var=$1; va=$2; vb=$3; n=${4:-3}
    for r in $(seq $n); do
      for v in $va $vb; do
        env $var=$v timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'$var':'$v','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" >> $O/ab.jsonl
      done
    done ;;
  step_trace)     # kernel trace + stats of the headline step, graph off and on
    export TMPDIR=/tmp
    for gr in off on; do
      timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/$gr -o step --output-format csv -- \
        python3 bench.py --steps 10 --warmup 3 --graph $gr > $O/bench_$gr.json 2> $O/bench_$gr.err || { tail -20 $O/bench_$gr.err; exit 1; }
    done ;;
  pmc_step)       # per-kernel counters of the headline step (graph off): two passes, each within
                  # the per-block slot limits (8 SQ, 4 TCC, 2 GRBM), then one merged summary
    export TMPDIR=/tmp
    timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_VALU_MFMA_BUSY_CYCLES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_BUSY_CYCLES TCC_HIT_sum TCC_MISS_sum \
      -d $O/p1 -o step --output-format csv -- python3 bench.py --steps 3 --warmup 2 --graph off > $O/p1.log 2>&1 || { tail -20 $O/p1.log; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAIT_INST_LDS \
      -d $O/p2 -o step --output-format csv -- python3 bench.py --steps 3 --warmup 2 --graph off > $O/p2.log 2>&1 || { tail -20 $O/p2.log; exit 1; }
    python3 -m vi_normflows_amd.bench.pmc_summary $O/p1 $O/p2 > $O/summary.txt && cat $O/summary.txt ;;
  iaf_graph)      # IAF engine: eager vs graph-replayed forward + backward, buffer by buffer; a
                  # test failure is data here (the chain continues), a hang / fault is not
    timeout -k 10 300 python -u -m pytest tests/test_iaf_engine.py -m gpu -k graph -v --timeout 240 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1
    rc=$?; grep -E "PASS|FAIL|assert|differs|Error" $O/pytest.txt | head -20
    [ $rc -le 1 ] || exit $rc ;;
  wg_pitch)       # weight-gradient launch vs operand row pitch (power of two or padded), both
                  # kernels, plus the L2 counters of the 4-wave one at each pitch
    for r in 1 2; do
      for pad in 0 64 32; do
        timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag pad$pad --layout-probe --layers 13 --iters 3 --layouts 0,3 --pitch-pad $pad >> $O/layout.jsonl || exit 1
      done
    done
    cat $O/layout.jsonl ;;
  wg_drift)       # L2 reuse of the 4-wave weight-gradient launch vs K (= batch): counters per K
    export TMPDIR=/tmp
    for b in 8192 32768 65536; do
      timeout -s KILL 240 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum \
        -d $O/pmc_b$b -o wg --output-format csv -- python3 -m vi_normflows_amd.bench.wgrad_bench --layers 13 --iters 1 --batch $b > $O/pmc_b$b.log 2>&1 || { tail -20 $O/pmc_b$b.log; exit 1; }
    done
    python3 - <<'PY'
import csv, collections, os
for b in (8192, 32768, 65536):
    f = f"gpurun_out/exp_wg_drift/pmc_b{b}/wg_counter_collection.csv"
    tot = collections.defaultdict(float); n = set()
    for r in csv.DictReader(open(f)):
        if "tn4w" not in r["Kernel_Name"]: continue
        tot[r["Counter_Name"]] += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
    h, m = tot["TCC_HIT_sum"], tot["TCC_MISS_sum"]
    rd, r128 = tot["TCC_EA0_RDREQ_sum"], tot["TCC_EA0_RDREQ_128B_sum"]
    eab = (128 * r128 + 64 * (rd - r128)) / max(len(n), 1)
    req = 256 * 2 * 256 * 2 * b
    print(b, "dispatches", len(n), "L2 hit %.3f" % (h / (h + m)), "fabric/requested %.3f" % (eab / req))
PY
    ;;
  wg_kchunk)      # timing probe: the weight-gradient launch as 1 / 2 / 4 / 8 K-chunk launches
    for r in 1 2; do
      for kc in 1 2 4 8; do
        timeout -k 10 300 python -m vi_normflows_amd.bench.wgrad_bench --tag kc$kc --layout-probe --layers 13 --iters 3 --layouts 3 --kchunks $kc >> $O/layout.jsonl || exit 1
      done
    done
    cat $O/layout.jsonl ;;
  var_ab)         # a variant library (arg: name) vs default: its GEMM / engine tests, the bf16
                  # products, and 3 alternating whole-step runs
    v=$1; P=vi_normflows_amd/_native/libvinf_hip_$v.so
    VINF_NATIVE_LIB=$P timeout -k 10 300 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_persistent_gpu.py tests/test_realnvp_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest_$v.txt 2>&1 || { tail -30 $O/pytest_$v.txt; exit 1; }
    tail -1 $O/pytest_$v.txt
    for r in 1 2; do
      timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --tag default --iters 20 --only fwd_l1,fwd_l2,dgrad_l3,dgrad_l2 >> $O/sg.jsonl || exit 1
      VINF_NATIVE_LIB=$P timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --tag $v --iters 20 --only fwd_l1,fwd_l2,dgrad_l3,dgrad_l2 >> $O/sg.jsonl || exit 1
    done
    for r in 1 2 3; do
      for lib in default $v; do
        if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$P; fi
        timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" >> $O/bench.jsonl
      done
    done
    unset VINF_NATIVE_LIB
    grep -v sum $O/sg.jsonl; cat $O/bench.jsonl ;;
  tests)          # selected GPU test files: args "<pytest paths / -k expr>" [tag]
    tag=${2:-t}
    timeout -k 10 900 python -u -m pytest $1 -m gpu -x -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/$tag.txt 2>&1 || { tail -40 $O/$tag.txt; exit 1; }
    tail -3 $O/$tag.txt ;;
  tests_all)      # as "tests" but every test runs (failures are listed, the chain continues
                  # unless the run hung or crashed)
    tag=${2:-t}
    timeout -k 10 900 python -u -m pytest $1 -m gpu -q --timeout 240 --timeout-method thread -p no:cacheprovider > $O/$tag.txt 2>&1
    rc=$?; tail -12 $O/$tag.txt; [ $rc -le 1 ] || exit $rc ;;
  dp_contention)  # RCCL CU-occupancy emulation on the headline step (bench/dp_contention.py)
    timeout -k 10 600 python -m vi_normflows_amd.bench.dp_contention "$@" > $O/dpc.jsonl 2> $O/dpc.err || { tail -20 $O/dpc.err; exit 1; }
    cat $O/dpc.jsonl ;;
  bench)          # headline bench on this box: args [tag] [extra bench args]
    tag=${1:-base}; shift
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 "$@" > $O/$tag.json 2> $O/$tag.err || { tail -20 $O/$tag.err; exit 1; }
    python -c "import json;d=json.load(open('$O/$tag.json'));print('BENCH $tag', d['ms_per_step'], d['value'], d['notes']['final_free_energy'])" ;;
  roofline)       # per-family HBM bytes / MFMA roofline of a step (bench/roofline.py): two counter
                  # passes (EA read requests by size + MFMA; EA write requests + L2 hit/miss) and an
                  # un-profiled kernel trace of the same command. args: TAG [bench / configs args]
    export TMPDIR=/tmp
    tag=${1:-step}; shift
    cmd="python3 bench.py --steps 3 --warmup 2 --graph off"; model="--model realnvp32"
    if [ $# -gt 0 ]; then cmd="python3 -m vi_normflows_amd.bench.configs --graph off --steps 3 --warmup 2 $*"; model=""; fi
    R=$O/$tag; mkdir -p $R
    timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_128B_sum TCC_EA0_RDREQ_32B_sum GRBM_GUI_ACTIVE SQ_INSTS_MFMA SQ_VALU_MFMA_BUSY_CYCLES \
      -d $R/rd -o step --output-format csv -- $cmd > $R/rd.log 2>&1 || { tail -20 $R/rd.log; exit 1; }
    timeout -s KILL 240 rocprofv3 --pmc TCC_EA0_WRREQ_sum TCC_EA0_WRREQ_64B_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE \
      -d $R/wr -o step --output-format csv -- $cmd > $R/wr.log 2>&1 || { tail -20 $R/wr.log; exit 1; }
    timeout -k 10 240 rocprofv3 --kernel-trace --stats -d $R/trace -o step --output-format csv -- $cmd > $R/trace.log 2>&1 || { tail -20 $R/trace.log; exit 1; }
    python3 -m vi_normflows_amd.bench.roofline --pmc $R/rd $R/wr --trace $R/trace --steps 0 $model > $R/roofline.txt && cat $R/roofline.txt ;;
  configs)        # north-star config refresh on the current tree (one line per run)
    for args in "--config 0 --batch 128" "--config 0 --batch 1024" "--config 2 --batch 32768" "--config 2 --batch 65536" \
                "--config 4 --batch 8192" "--config 4 --batch 32768" "--config 5 --precision bf16 --batch 32768" "--config 5 --precision fp8 --batch 32768" \
                "--config 5 --precision bf16 --batch 32768" "--config 5 --precision fp8 --batch 32768"; do
      timeout -k 10 240 python -m vi_normflows_amd.bench.configs $args >> $O/configs.jsonl 2>> $O/configs.err || { echo "FAIL $args"; tail -20 $O/configs.err; exit 1; }
    done ;;
  lib_ab_cfg5)    # default library vs a variant build (arg: variant name): GEMM tests on the
                  # default, then per-product, headline and config-5 timings, alternating
    v=$1; L=vi_normflows_amd/_native/libvinf_hip_$v.so
    timeout -k 10 600 python -u -m pytest tests/test_gemm_gpu.py tests/test_gemm_persistent_gpu.py tests/test_realnvp_engine.py tests/test_maf_engine.py -m gpu -x -q --timeout 120 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -30 $O/pytest.txt; exit 1; }
    tail -1 $O/pytest.txt
    for r in 1 2; do
      for lib in default $v; do
        if [ $lib = default ]; then unset VINF_NATIVE_LIB; else export VINF_NATIVE_LIB=$L; fi
        timeout -k 10 120 python -m vi_normflows_amd.bench.step_gemms --tag $lib --iters 20 --only fwd_l2,cpl_fwd,dgrad_l2,cpl_bwd >> $O/sg.jsonl || exit 1
        timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" >> $O/bench.jsonl
        for pr in bf16 fp8; do
          timeout -k 10 240 python -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch 32768 > $O/c.json 2>> $O/c.err || { tail -20 $O/c.err; exit 1; }
          python -c "import json;d=json.load(open('$O/c.json'));print(json.dumps({'lib':'$lib','prec':'$pr','ms':d['ms_per_step'],'sps':d['samples_per_s']}))" >> $O/cfg5.jsonl
        done
      done
    done
    unset VINF_NATIVE_LIB ;;
  step_libs)      # whole headline step, this tree's library vs variant builds, interleaved
                  # (args: [rounds] variants...)
    n=$1; shift
    for r in $(seq $n); do
      for lib in default "$@"; do
        if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
        VINF_NATIVE_LIB=$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'lib':'$lib','ms':d['ms_per_step'],'F':d['notes']['final_free_energy']}))" | tee -a $O/bench.jsonl
      done
    done ;;
  cfg5_libs)      # config 5 (MAF-64, B = 32768) fp8 and bf16, this tree's library vs variants
                  # (args: [rounds] variants...)
    n=$1; shift
    for r in $(seq $n); do
      for lib in default "$@"; do
        if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
        for pr in fp8 bf16; do
          VINF_NATIVE_LIB=$L timeout -k 10 240 python -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch 32768 > $O/c.json 2>> $O/c.err || { tail -20 $O/c.err; exit 1; }
          python -c "import json;d=json.load(open('$O/c.json'));print(json.dumps({'lib':'$lib','prec':'$pr','ms':d['ms_per_step'],'sps':d['samples_per_s']}))" | tee -a $O/cfg5.jsonl
        done
      done
    done ;;
  sg_ab)          # per-product step-GEMM timings, default library vs variant builds
                  # (args: "<products>" variants...; e.g. "fwd_l2,cpl_fwd,dgrad_l2" spread2)
    ONLY=$1; shift
    for r in 1 2; do
      for v in default "$@"; do
        if [ $v = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$v.so; fi
        VINF_NATIVE_LIB=$L timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --tag $v --iters 20 --only $ONLY >> $O/sg.jsonl 2> $O/sg_$v.err || { tail -20 $O/sg_$v.err; exit 1; }
      done
    done
    grep -v '"sum"' $O/sg.jsonl ;;
  quick)          # selected GPU tests, per-product timings, headline bench
                  # (args: "<pytest paths>" ["<step_gemms --only list>"])
    TESTS=$1; ONLY=${2:-fwd_l1,fwd_l2,fwd_l2_nomask,cpl_fwd,dgrad_l3,dgrad_l2,cpl_bwd}
    if [ -n "$TESTS" ]; then
      timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
      tail -2 $O/pytest.txt
    fi
    timeout -k 10 180 python -m vi_normflows_amd.bench.step_gemms --iters 20 --only $ONLY > $O/sg.jsonl 2> $O/sg.err || { echo SG_FAIL; tail -20 $O/sg.err; exit 1; }
    cat $O/sg.jsonl
    timeout -k 10 240 python bench.py --steps 20 --warmup 5 > $O/bench.json 2> $O/bench.err || { echo BENCH_FAIL; tail -20 $O/bench.err; exit 1; }
    python -c "import json;d=json.load(open('$O/bench.json'));print('BENCH', d['ms_per_step'], d['value'], d['notes']['final_free_energy'])" ;;
  cfg_trace)      # kernel trace of one north-star config (graph off): args CONFIG BATCH [configs.py args]
    export TMPDIR=/tmp
    c=$1; b=$2; shift 2
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_$c -o run --output-format csv -- \
      python3 -m vi_normflows_amd.bench.configs --config $c --batch $b --graph off --steps 5 --warmup 3 "$@" > $O/r_$c.json 2> $O/r_$c.err || { tail -20 $O/r_$c.err; exit 1; }
    python3 -m vi_normflows_amd.bench.prof_summary $O/t_$c > $O/summary_$c.txt 2>&1; head -20 $O/summary_$c.txt; cat $O/r_$c.json ;;
  configs_final)  # every north-star config once, engine and module paths (one process each)
    for args in "--config 0 --batch 128" "--config 0 --batch 1024" "--config 0 --impl module --batch 1024" \
                "--config 2 --batch 32768" "--config 3 --batch 16384" \
                "--config 4 --batch 8192" "--config 4 --impl module --batch 8192" \
                "--config 5 --precision bf16 --batch 32768" "--config 5 --precision fp8 --batch 32768"; do
      timeout -k 10 300 python -m vi_normflows_amd.bench.configs $args >> $O/configs.jsonl 2>> $O/configs.err || { echo "FAIL $args"; tail -20 $O/configs.err; exit 1; }
      tail -1 $O/configs.jsonl | cut -c1-300
    done ;;
  f8_ab)          # config-5 fp8 vs bf16, interleaved (args: [batch] [rounds]) after the fp8 tests
    b=${1:-32768}; n=${2:-2}
    timeout -k 10 400 python -u -m pytest tests/test_fp8_wgrad_gpu.py tests/test_maf_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { tail -40 $O/pytest.txt; exit 1; }
    tail -1 $O/pytest.txt
    for r in $(seq $n); do
      for pr in fp8 bf16; do
        timeout -k 10 240 python -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch $b >> $O/cfg5.jsonl 2>> $O/cfg5.err || { tail -20 $O/cfg5.err; exit 1; }
      done
    done
    python -c "
import json
for l in open('$O/cfg5.jsonl'):
    d=json.loads(l); print(d.get('precision'), d.get('ms_per_step'), d.get('samples_per_s'))" ;;
  rccl_trace)     # kernel traces of the headline step, plain graph path vs the 1-rank RCCL path
                  # (bench.py --force-reduce [args]) on one box
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/plain -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 > $O/plain.log 2>&1 || { echo PLAIN_FAIL; tail -20 $O/plain.log; exit 1; }
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/rccl -o step --output-format csv -- python3 bench.py --steps 10 --warmup 3 --force-reduce "$@" > $O/rccl.log 2>&1 || { echo RCCL_FAIL; tail -20 $O/rccl.log; exit 1; }
    for t in plain rccl; do
      python3 -m vi_normflows_amd.bench.prof_summary $O/$t > $O/${t}_summary.txt 2>&1
      python3 -m vi_normflows_amd.bench.gap_summary $O/$t > $O/${t}_gaps.txt 2>&1 || true
    done
    head -14 $O/plain_summary.txt; head -24 $O/rccl_summary.txt ;;
  cfg_trace_libs) # kernel traces of one north-star config on this tree's library and on variant
                  # builds (probe builds included: timings only): args CONFIG BATCH PREC variants...
    export TMPDIR=/tmp
    c=$1; b=$2; pr=$3; shift 3
    for lib in default "$@"; do
      if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
      VINF_NATIVE_LIB=$L timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_${lib}_$pr -o run --output-format csv -- \
        python3 -m vi_normflows_amd.bench.configs --config $c --batch $b --precision $pr --graph off --steps 5 --warmup 3 > $O/r_${lib}_$pr.json 2> $O/r_${lib}_$pr.err || { tail -20 $O/r_${lib}_$pr.err; exit 1; }
      python3 -m vi_normflows_amd.bench.prof_summary $O/t_${lib}_$pr > $O/summary_${lib}_$pr.txt 2>&1
      echo "== $lib $pr"; head -8 $O/summary_${lib}_$pr.txt
    done ;;
  f8_lib_ab)      # e4m3 path of a variant build (arg: V): the fp8 / MAF GPU tests on V, the
                  # e4m3 256x256 products alternating default / V, config-5 fp8 kernel traces and
                  # two interleaved config-5 rounds (fp8 and bf16)
    v=$1; P=vi_normflows_amd/_native/libvinf_hip_$v.so
    VINF_NATIVE_LIB=$P timeout -k 10 600 python -u -m pytest tests/test_fp8_gpu.py tests/test_fp8_wgrad_gpu.py tests/test_maf_engine.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
    tail -1 $O/pytest.txt
    for lib in default $v default $v; do
      if [ $lib = default ]; then L=""; else L=$P; fi
      VINF_NATIVE_LIB=$L timeout -k 10 200 python -m vi_normflows_amd.bench.gemm_bench --batch 32768 --only fwd_l2_fp8,sq4096_fp8 > $O/g.txt 2>&1 || { tail -20 $O/g.txt; exit 1; }
      grep shape $O/g.txt | sed "s/^/$lib /" | tee -a $O/gemm.txt
    done
    bash scripts/experiments.sh cfg_trace_libs 5 32768 fp8 $v && bash scripts/experiments.sh cfg5_libs 2 $v ;;
  cfg5_state_ab)  # config 5 with the bf16 MAF state (KernelPaths.maf_bf16_state) vs the fp32
                  # state: the MAF engine GPU tests, then interleaved fp8 / bf16 runs [rounds] and
                  # an fp8 kernel trace with the option
    export TMPDIR=/tmp
    timeout -k 10 600 python -u -m pytest tests/test_maf_engine.py -m gpu -x -q -s --timeout 300 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -40 $O/pytest.txt; exit 1; }
    grep "bf16 state\|passed" $O/pytest.txt
    for r in $(seq ${1:-2}); do
      for st in 0 1; do
        for pr in fp8 bf16; do
          VINF_KERNEL_PATHS=maf_bf16_state=$st timeout -k 10 240 python -m vi_normflows_amd.bench.configs --config 5 --precision $pr --batch 32768 > $O/c.json 2>> $O/c.err || { tail -20 $O/c.err; exit 1; }
          python -c "import json;d=json.load(open('$O/c.json'));print(json.dumps({'bf16_state':$st,'prec':'$pr','ms':d['ms_per_step'],'sps':d['samples_per_s']}))" | tee -a $O/cfg5.jsonl
        done
      done
    done
    VINF_KERNEL_PATHS=maf_bf16_state=1 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/t_state -o run --output-format csv -- \
      python3 -m vi_normflows_amd.bench.configs --config 5 --batch 32768 --precision fp8 --graph off --steps 5 --warmup 3 > $O/r_state.json 2> $O/r_state.err || { tail -20 $O/r_state.err; exit 1; }
    python3 -m vi_normflows_amd.bench.prof_summary $O/t_state > $O/summary_state.txt 2>&1; head -10 $O/summary_state.txt ;;
  f8_pmc)         # wave-state counters of the 256x256 kernel on the 4096^3 product, bf16 vs e4m3
                  # (args: [variant libs]): where an e4m3 K-tile spends its extra time
    export TMPDIR=/tmp
    P1="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_MFMA"
    P2="GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_VMEM SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_ACTIVE_INST_MISC"
    for lib in default "$@"; do
      if [ $lib = default ]; then L=""; else L=vi_normflows_amd/_native/libvinf_hip_$lib.so; fi
      for s in sq4096 sq4096_fp8; do
        for pp in 1 2; do
          eval "C=\$P$pp"
          VINF_NATIVE_LIB=$L timeout -s KILL 120 rocprofv3 --pmc $C -d $O/${lib}_${s}_p$pp -o pmc --output-format csv -- python3 -m vi_normflows_amd.bench.gemm_bench --only $s > $O/${lib}_${s}_p$pp.log 2>&1 || { echo P${pp}_FAIL $lib $s; tail -20 $O/${lib}_${s}_p$pp.log; exit 1; }
        done
        python3 -m vi_normflows_amd.bench.pmc_summary $O/${lib}_${s}_p1 $O/${lib}_${s}_p2 > $O/${lib}_${s}_summary.txt 2>&1
        echo "== $lib $s"; cat $O/${lib}_${s}_summary.txt
      done
    done ;;
  rccl_ab)        # the 1-rank RCCL path (bench.py --force-reduce) of this tree's library vs a
                  # variant build, with the plain step alongside: args V [rounds]; the persistent
                  # GEMM GPU tests first
    v=$1; r=${2:-3}; P=vi_normflows_amd/_native/libvinf_hip_$v.so
    timeout -k 10 400 python -u -m pytest tests/test_gemm_persistent_gpu.py -m gpu -x -q --timeout 200 --timeout-method thread -p no:cacheprovider > $O/pytest.txt 2>&1 || { echo PYTEST_FAIL; tail -30 $O/pytest.txt; exit 1; }
    tail -1 $O/pytest.txt
    for i in $(seq $r); do
      for arm in plain rccl rccl_$v; do
        L=""; X=""
        [ $arm != plain ] && X=--force-reduce
        [ $arm = rccl_$v ] && L=$P
        VINF_NATIVE_LIB=$L timeout -k 10 240 python bench.py --steps 20 --warmup 5 $X > $O/b.json 2> $O/b.err || { echo BENCH_FAIL; tail -20 $O/b.err; exit 1; }
        python -c "import json;d=json.load(open('$O/b.json'));print(json.dumps({'arm':'$arm','ms':d['ms_per_step'],'identical':d['notes']['replicas_identical']}))" | tee -a $O/ab.jsonl
      done
    done ;;
  getdata_trace)  # kernel trace of the 2-D potential CLI on the GPU (fused target kernel)
    export TMPDIR=/tmp
    timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 -m vi_normflows_amd.get_data 8 100 0.02 p1 --device cuda --samples 1048576 --quiet > $O/out.txt 2>&1 || { echo PROF_FAIL; tail -20 $O/out.txt; exit 1; }
    tail -3 $O/out.txt
    python3 -m vi_normflows_amd.bench.prof_summary $O/prof > $O/summary.txt 2>&1 && head -25 $O/summary.txt ;;
  *) echo "unknown experiment $name"; exit 2 ;;
esac
