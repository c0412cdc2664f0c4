#!/bin/bash
# r06 GPU runner: STEPS picks what runs (space-separated):
#   smoke      __graft_entry__.smoke()
#   large      tests/test_gpu_large.py (the 2 GiB+ squares and the wide forms)
#   tests      every -m gpu test
#   bench      the default bench.py line
#   headline   rocprofv3 stats of the headline launch
#   pmc        FETCH_SIZE / WRITE_SIZE passes of the headline launch
# RUN names the output directory under gpurun_out/.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${RUN:-r06}; mkdir -p $OUT
export TMPDIR=/tmp
step() { local n=$1 t=$2; shift 2; echo "[$(date +%T)] $n" >> $OUT/steps.log; timeout -k 10 $t "$@" > $OUT/$n.log 2>&1; local rc=$?; echo "[$(date +%T)] $n rc=$rc" >> $OUT/steps.log; tail -n 4 $OUT/$n.log; return $rc; }
for s in ${STEPS:-smoke tests}; do
  case $s in
    smoke) step smoke 300 python3 -c "import __graft_entry__ as g; g.smoke()" || exit 3 ;;
    large) step large 900 python3 -u -m pytest tests/test_gpu_large.py -m gpu -v -x --timeout 300 --timeout-method thread || exit 4 ;;
    tests) step pytest_gpu 1000 python3 -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread || exit 5 ;;
    bench) step bench 700 python3 bench.py || exit 6 ;;
    headline) step prof 300 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/prof" -o run --output-format csv -- python3 bench.py --headline-only --steps 50 || exit 7 ;;
    pmc) step pmc_fetch 300 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/pmc_fetch" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 8
         step pmc_write 300 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/pmc_write" -o run --output-format csv -- python3 bench.py --headline-only --steps 3 --warmup 1 || exit 9
         python3 scripts/pmc_summary.py $OUT/pmc_fetch $OUT/pmc_write $OUT/pmc_latest.json > $OUT/pmc_summary.log 2>&1 ;;
    gf16pmc)  # counters of the production GF(2^16) encoders (c4 k=256 S=2048, c5 k=512 S=512)
         i=0
         for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
                  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
                  "SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"; do
           i=$((i+1))
           step gf16_sq$i 120 rocprofv3 --pmc $C -d "$PWD/$OUT/gf16_sq$i" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 3 || exit 10
         done
         step gf16_fetch 120 rocprofv3 --pmc FETCH_SIZE -d "$PWD/$OUT/gf16_fetch" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 3 || exit 11
         step gf16_write 120 rocprofv3 --pmc WRITE_SIZE -d "$PWD/$OUT/gf16_write" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 3 || exit 12
         step gf16_stats 120 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/gf16_prof" -o run --output-format csv -- python3 scripts/diag/run_gf16.py 20 || exit 13
         python3 scripts/sq_summary.py $OUT/gf16_sq.json $OUT/gf16_sq1 $OUT/gf16_sq2 $OUT/gf16_sq3 > $OUT/gf16_sq_summary.log 2>&1
         python3 scripts/pmc_summary.py $OUT/gf16_fetch $OUT/gf16_write $OUT/gf16_pmc.json > $OUT/gf16_pmc_summary.log 2>&1 ;;
    decab) DECAB_KS=${DECAB_KS:-128,256,512} DECAB_V8=${DECAB_V8:-0,1} DECAB_V16=${DECAB_V16:-0} \
             step decab 300 python3 scripts/diag/dec_ab.py || exit 14 ;;
    gf16ab) GF16AB_FORMS=${GF16AB_FORMS:-0} GF16AB_C4FORMS=${GF16AB_C4FORMS:-0,20} GF16AB_REPS=${GF16AB_REPS:-3} \
             step gf16ab 300 python3 scripts/diag/gf16_ab.py || exit 15 ;;
    repairtrace) step repair_trace 300 rocprofv3 --kernel-trace --memory-copy-trace -d "$PWD/$OUT/rtrace" -o run --output-format csv -- python3 scripts/diag/repair_trace.py ${RT_REPS:-6} || exit 16 ;;
    repab) step repair_ab 400 python3 scripts/diag/repair_ab.py || exit 17 ;;
    singlepmc)  # counters of the single-square latency form (encode_gf8_split16_kernel since r06p)
         i=0
         for C in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_ACTIVE_INST_VALU" \
                  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_LDS_BANK_CONFLICT SQ_ACTIVE_INST_SCA" \
                  "SQ_INST_LEVEL_VMEM SQ_INSTS_SMEM SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"; do
           i=$((i+1))
           step single_sq$i 120 rocprofv3 --pmc $C -d "$PWD/$OUT/single_sq$i" -o run --output-format csv -- python3 scripts/diag/run_single.py 20 || exit 21
         done
         step single_stats 120 rocprofv3 --kernel-trace --stats -d "$PWD/$OUT/single_prof" -o run --output-format csv -- python3 scripts/diag/run_single.py 200 || exit 22
         python3 scripts/sq_summary.py $OUT/single_sq.json $OUT/single_sq1 $OUT/single_sq2 $OUT/single_sq3 > $OUT/single_sq_summary.log 2>&1 ;;
    decfloor) DECAB_KS=128 DECAB_V8=${DECAB_V8:-0,2,1} step decfloor 300 python3 scripts/diag/dec_ab.py || exit 23 ;;
    gf8ab)  # GF(2^8) byte-table kernels: this build's diagnostic library against librsmt2d_hip_diag_ab.so
         for rep in 1 2; do
           for lib in rsmt2d_amd/librsmt2d_hip_diag.so rsmt2d_amd/librsmt2d_hip_diag_ab.so; do
             RSM_DIAG_LIB=$lib step gf8ab_$(basename $lib .so)_$rep 300 python3 scripts/diag/gf8_ab.py || exit 24
           done
         done ;;
    repab2)  # Repair (zero-copy sweeps): this build's diagnostic library against librsmt2d_hip_diag_ab.so
         for rep in 1 2; do
           for lib in rsmt2d_amd/librsmt2d_hip_diag.so rsmt2d_amd/librsmt2d_hip_diag_ab.so; do
             RSM_DIAG_LIB=$lib REPAB_KS=${REPAB_KS:-128,256,512} step repab_$(basename $lib .so)_$rep 300 python3 scripts/diag/repair_ab.py || exit 25
           done
         done ;;
    gf16ab2)  # GF(2^16) encoder forms (GF16AB_FORMS / GF16AB_C4FORMS): this build's diagnostic library
              # against librsmt2d_hip_diag_ab.so
         for rep in 1 2; do
           for lib in rsmt2d_amd/librsmt2d_hip_diag.so rsmt2d_amd/librsmt2d_hip_diag_ab.so; do
             RSM_DIAG_LIB=$lib GF16AB_FORMS=${GF16AB_FORMS:-0,21} GF16AB_C4FORMS=${GF16AB_C4FORMS:-0,21} GF16AB_REPS=2 \
               step gf16ab2_$(basename $lib .so)_$rep 300 python3 scripts/diag/gf16_ab.py || exit 26
           done
         done ;;
    lutprobe) step lutprobe 120 scripts/diag/lutprobe ${LUT_ITERS:-4096} || exit 18 ;;
    selab)  # same-box A/B of the production GF(2^16) kernels: this build's diagnostic library
            # against the variant build librsmt2d_hip_diag_ab.so (make ab AB_FLAGS=...)
         for rep in 1 2; do
           for lib in rsmt2d_amd/librsmt2d_hip_diag.so rsmt2d_amd/librsmt2d_hip_diag_ab.so; do
             tag=$(basename $lib .so)
             RSM_DIAG_LIB=$lib GF16AB_FORMS=0 GF16AB_C4FORMS=0 GF16AB_REPS=2 step gf16ab_${tag}_$rep 300 python3 scripts/diag/gf16_ab.py || exit 19
             RSM_DIAG_LIB=$lib DECAB_KS=${SELAB_KS:-256,512} DECAB_V16=0 step decab_${tag}_$rep 300 python3 scripts/diag/dec_ab.py || exit 20
           done
         done ;;
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
