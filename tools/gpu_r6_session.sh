#!/bin/bash
# Round-6 focused GPU session.  Usage: <tag> <step>...  Steps (each under its own time limit,
# stop at the first failure):
#   valtests   the validator / path GPU tests
#   valab      validator file path A/B: the in-tree library vs tools/ablib/val_r5.so (round 5's
#              whole-file pread windows), interleaved, 2,000 tmpfs files, 6 passes each
#   valab2     the same over several builds: in-tree + $VAL_VARIANTS (tools/ablib/<name>.so)
#   h2d        tools/h2d_sizes.py: H2D rate by transfer size, one and two streams
#   mmapprobe  tools/probe_mmap_reg (needs it built): tmpfs files mapped + hipHostRegister'ed, DMA'd
#              straight to HBM, vs the pread copy
#   probe      tools/probe_pread (needs it built) twice: the file path's reads by destination form
#   numa       the gather pool bound to the GPU's NUMA node (default) vs unbound (SD_CAS_POOL_NUMA=0):
#              the validator file path (3 rounds) and config 1 (2 rounds)
#   c1ab       config 1 on the in-tree build vs $C1_VARIANTS (tools/ablib/<name>.so), 3 rounds
#   config1    BASELINE config 1 with 7 timed drop-in passes, twice, then one traced pass
#   reh2 reh4  the one-GPU rehearsals of the N = 2 / N = 4 bench lines
#   sorttests  the sort / grouping / link GPU tests
#   sortab     LSD grouping at 12.5 M keys: in-tree vs $SORT_VARIANTS (default sort_r5: round
#              5's group.hip), 3 interleaved rounds, then a rocprofv3 kernel trace of the new one
#   sortpmc    tools/gpu_r6_pmc_sort.sh (HBM bytes per key of hash / lsd / lsdapi)
#   power      tools/power_split.py (needs tools/ubench_k1 built): where K1's random-content power goes
#   stress     randomised parity: grouping with the forced LSD path every iteration, link
#              emission vs the replay, the path gather + validator file path vs the C oracle
#   powerab    K1 on random content, product layout vs the 64-file LINE / QUAD tiled layouts,
#              10 s sustained each, 3 rounds (the HBM-energy lever)
#   sortstall  SQ stall / instruction counters of the LSD grouping's kernels (two rocprofv3 --pmc passes)
#   stresslong longer randomised stress on the final code (~15 min)
#   repeat     the default `python bench.py` and the validator file path twice, on another box
#   valshapes  the validator file path on 20,000 small files, 150 files of 16-60 MiB, and 40 files
#              of 128-192 MiB (streamed one by one)
#   streamab   the streamed single-file path (40 files of 128-192 MiB; one 4 GiB file): in-tree vs
#              $STREAM_VARIANTS, 2 rounds
#   smalltrace the validator file path on 20,000 small files with SD_CAS_TRACE=1
#   suite      the whole GPU suite (release)
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r6}
shift
mkdir -p $OUT
cd $R
for step in "$@"; do
  case $step in
    valtests)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "checksum or from_paths or host_pool" > $OUT/pytest_validator.log 2>&1 || { echo VALTESTS_FAIL; tail -30 $OUT/pytest_validator.log; exit 1; }
      tail -1 $OUT/pytest_validator.log ;;
    valab)
      for k in 1 2; do
        timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/val_new_$k.log 2>&1 || { echo VALAB_FAIL; tail -20 $OUT/val_new_$k.log; exit 1; }
        SD_HIP_CAS_LIB=$R/tools/ablib/val_r5.so timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/val_r5_$k.log 2>&1 || { echo VALAB_FAIL; tail -20 $OUT/val_r5_$k.log; exit 1; }
      done
      SD_CAS_TRACE=1 timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 4 > $OUT/val_new_trace.log 2>&1 || { echo VALAB_FAIL; exit 1; }
      grep -h '"files"' $OUT/val_*_[12].log | cut -c1-400 ;;
    valab2)
      for k in $(seq 1 ${VAL_ROUNDS:-2}); do
        for v in intree ${VAL_VARIANTS:-val_r5}; do
          lib=""; [ $v != intree ] && lib=$R/tools/ablib/$v.so
          SD_HIP_CAS_LIB=$lib timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/val2_${v}_$k.log 2>&1 || { echo VALAB2_FAIL; tail -20 $OUT/val2_${v}_$k.log; exit 1; }
        done
      done ;;
    h2d)
      timeout -k 10 200 python3 -u tools/h2d_sizes.py > $OUT/h2d_sizes.log 2>&1 || { echo H2D_FAIL; tail -20 $OUT/h2d_sizes.log; exit 1; } ;;
    mmapprobe)
      timeout -k 10 300 tools/probe_mmap_reg 15 > $OUT/probe_mmap_reg.log 2>&1 || { echo MMAP_FAIL; tail -20 $OUT/probe_mmap_reg.log; exit 1; }
      cat $OUT/probe_mmap_reg.log ;;
    probe)
      for k in 1 2; do
        timeout -k 10 300 tools/probe_pread 15 $R/spacedrive_amd/libsd_hip_cas.so > $OUT/probe_pread_$k.log 2>&1 || { echo PROBE_FAIL; tail -20 $OUT/probe_pread_$k.log; exit 1; }
      done
      cat $OUT/probe_pread_*.log ;;
    fdsab)
      # the pool's private descriptor tables (SD_CAS_POOL_PRIVATE_FDS=1, the default) vs the
      # shared table: config 1 (the drop-in gather), the 2,000-file validator set, 20,000 small
      # files, interleaved
      for k in 1 2; do
        for m in 1 0; do
          SD_CAS_POOL_PRIVATE_FDS=$m SD_CONFIG1_PASSES=7 timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/config1fds${m}_$k.log 2>&1 || { echo FDSAB_FAIL; tail -20 $OUT/config1fds${m}_$k.log; exit 1; }
          SD_CAS_POOL_PRIVATE_FDS=$m timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/valfds${m}_$k.log 2>&1 || { echo FDSAB_FAIL; tail -20 $OUT/valfds${m}_$k.log; exit 1; }
          SD_CAS_POOL_PRIVATE_FDS=$m timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 20000 --path-kib 16 256 --path-runs 4 > $OUT/smallfds${m}_$k.log 2>&1 || { echo FDSAB_FAIL; tail -20 $OUT/smallfds${m}_$k.log; exit 1; }
        done
      done
      grep -h '"gpu_dropin_files_per_s"' $OUT/config1fds*.log | python3 -c "import sys,json; [print(json.loads(l).get('gpu_dropin_passes_files_per_s'), json.loads(l)['job_step_100_ms_median']) for l in sys.stdin]"
      grep -h '"files"' $OUT/valfds*.log $OUT/smallfds*.log | cut -c1-220 ;;
    hostab)
      # config 3 as worded (pinned host memory -> HBM -> K1): session 23's build split each
      # batch's copy in two halves over the two copy streams; hcs1 = one stream (the kept
      # form: no difference, the split is in git history), interleaved
      timeout -k 10 300 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread -k "sampled_host" > $OUT/pytest_host.log 2>&1 || { echo HOSTAB_FAIL; tail -30 $OUT/pytest_host.log; exit 1; }
      tail -1 $OUT/pytest_host.log
      for k in 1 2 3; do
        for v in intree hcs1; do
          lib=""; [ $v != intree ] && lib=$R/tools/ablib/$v.so
          SD_HIP_CAS_LIB=$lib timeout -k 10 300 python3 -u tools/bench_configs.py --config 3e > $OUT/c3e_${v}_$k.log 2>&1 || { echo HOSTAB_FAIL; tail -20 $OUT/c3e_${v}_$k.log; exit 1; }
        done
      done
      grep -h '"3-e2e"' $OUT/c3e_*.log | cut -c1-200 ;;
    numa)
      for k in 1 2 3; do
        for m in 1 0; do
          SD_CAS_POOL_NUMA=$m timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/valnuma${m}_$k.log 2>&1 || { echo NUMA_FAIL; tail -20 $OUT/valnuma${m}_$k.log; exit 1; }
        done
      done
      for k in 1 2; do
        for m in 1 0; do
          SD_CAS_POOL_NUMA=$m SD_CONFIG1_PASSES=7 timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/config1numa${m}_$k.log 2>&1 || { echo NUMA_FAIL; tail -20 $OUT/config1numa${m}_$k.log; exit 1; }
        done
      done
      SD_CAS_TRACE=1 timeout -k 10 120 python3 -u -c "from spacedrive_amd import CasEngine; CasEngine(0)" > $OUT/numa_ctx.log 2>&1 || { echo NUMA_FAIL; exit 1; }
      cat $OUT/numa_ctx.log ;;
    c1ab)
      for k in 1 2 3; do
        for v in intree ${C1_VARIANTS:-paths_caller}; do
          lib=""; [ $v != intree ] && lib=$R/tools/ablib/$v.so
          SD_HIP_CAS_LIB=$lib SD_CONFIG1_PASSES=7 timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/c1_${v}_$k.log 2>&1 || { echo C1AB_FAIL; tail -20 $OUT/c1_${v}_$k.log; exit 1; }
        done
      done ;;
    config1)
      for k in 1 2; do
        SD_CONFIG1_PASSES=7 timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/config1_$k.log 2>&1 || { echo CONFIG1_FAIL; tail -20 $OUT/config1_$k.log; exit 1; }
      done
      SD_CAS_TRACE=1 SD_CONFIG1_PASSES=7 timeout -k 10 300 python3 -u tools/bench_configs.py --config 1 > $OUT/config1_trace.log 2>&1 || { echo CONFIG1_FAIL; exit 1; }
      grep -h '"config"' $OUT/config1_[12].log | cut -c1-600 ;;
    reh2)
      SD_BENCH_ONE_DEVICE=1 SD_CPU_BASELINE_THREADS=16 timeout -k 10 500 python3 -u bench.py --gpus 2 --steps 10 --warmup 2 --files-per-gpu 262144 --e2e-files 1048576 > $OUT/bench_n2_rehearsal.log 2>&1 || { echo REH2_FAIL; tail -20 $OUT/bench_n2_rehearsal.log; exit 1; }
      tail -1 $OUT/bench_n2_rehearsal.log | cut -c1-300 ;;
    reh4)
      SD_BENCH_ONE_DEVICE=1 SD_CPU_BASELINE_THREADS=16 timeout -k 10 500 python3 -u bench.py --gpus 4 --steps 10 --warmup 2 --files-per-gpu 131072 --e2e-files 1048576 > $OUT/bench_n4_rehearsal.log 2>&1 || { echo REH4_FAIL; tail -20 $OUT/bench_n4_rehearsal.log; exit 1; }
      tail -1 $OUT/bench_n4_rehearsal.log | cut -c1-300 ;;
    sorttests)
      timeout -k 10 600 python3 -u -m pytest tests/test_gpu_parity.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread -k "sort or group or links or identifier" > $OUT/pytest_sort.log 2>&1 || { echo SORTTESTS_FAIL; tail -30 $OUT/pytest_sort.log; exit 1; }
      tail -1 $OUT/pytest_sort.log ;;
    sortab)
      for k in 1 2 3; do
        timeout -k 10 200 python3 -u tools/bench_group.py 1310720 12500000 > $OUT/group_new_$k.log 2>&1 || { echo SORTAB_FAIL; tail -20 $OUT/group_new_$k.log; exit 1; }
        for v in ${SORT_VARIANTS:-sort_r5}; do
          SD_HIP_CAS_LIB=$R/tools/ablib/$v.so timeout -k 10 200 python3 -u tools/bench_group.py --only lsd 12500000 > $OUT/group_${v}_$k.log 2>&1 || { echo SORTAB_FAIL; tail -20 $OUT/group_${v}_$k.log; exit 1; }
        done
      done
      grep -h '"keys": 12500000' $OUT/group_*_[123].log | cut -c1-300
      cd /tmp && export TMPDIR=/tmp
      timeout -k 10 200 rocprofv3 --kernel-trace --stats -d $OUT/sortprof -o run --output-format csv -- python3 $R/tools/bench_group.py --only lsd 12500000 > $OUT/sortprof.log 2>&1 || { echo SORTPROF_FAIL; exit 1; }
      cd $R ;;
    sortpmc)
      bash tools/gpu_r6_pmc_sort.sh ${OUT#$R/gpurun_out/}/pmc || { echo SORTPMC_FAIL; exit 1; } ;;
    power)
      timeout -k 10 400 python3 -u tools/power_split.py --seconds 6 --rounds 2 > $OUT/power_split.log 2>&1 || { echo POWER_FAIL; tail -20 $OUT/power_split.log; exit 1; }
      tail -1 $OUT/power_split.log ;;
    powerab)
      timeout -k 10 400 python3 -u tools/power_split.py --seconds 10 --rounds 3 --variants k1_rand,k1_line_rand,k1_quad_rand > $OUT/power_layout_ab.log 2>&1 || { echo POWERAB_FAIL; tail -20 $OUT/power_layout_ab.log; exit 1; }
      cat $OUT/power_layout_ab.log | cut -c1-250 ;;
    stress)
      timeout -k 10 300 python3 -u tools/stress_parity.py --seconds 150 --lsd-every 1 > $OUT/stress_parity_lsd.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_parity_lsd.log; exit 1; }
      tail -1 $OUT/stress_parity_lsd.log | cut -c1-300
      timeout -k 10 240 python3 -u tools/stress_links.py --seconds 90 > $OUT/stress_links.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_links.log; exit 1; }
      tail -1 $OUT/stress_links.log | cut -c1-300
      timeout -k 10 240 python3 -u tools/stress_paths.py --checksums --seconds 90 > $OUT/stress_paths.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_paths.log; exit 1; }
      tail -1 $OUT/stress_paths.log | cut -c1-300 ;;
    sortstall)
      i=0
      for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT" "SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD GRBM_GUI_ACTIVE GRBM_COUNT"; do
        i=$((i+1))
        (cd /tmp && export TMPDIR=/tmp && timeout -s KILL 90 rocprofv3 --kernel-trace --pmc $grp -d $OUT/sortstall/p$i -o run --output-format csv -- python3 $R/tools/bench_group.py --only lsd 12500000 > $OUT/sortstall_p$i.log 2>&1) || { echo "SORTSTALL_FAIL $i"; tail -5 $OUT/sortstall_p$i.log; exit 1; }
      done
      python3 tools/pmc_summarize.py $OUT/sortstall > $OUT/sortstall.json && echo SORTSTALL_OK ;;
    stresslong)
      timeout -k 10 420 python3 -u tools/stress_parity.py --seconds 300 --lsd-every 2 --validator > $OUT/stress_parity_long.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_parity_long.log; exit 1; }
      timeout -k 10 300 python3 -u tools/stress_parity.py --seconds 200 --fused --seed 77 > $OUT/stress_fused_long.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_fused_long.log; exit 1; }
      timeout -k 10 300 python3 -u tools/stress_links.py --seconds 180 --seed 11 > $OUT/stress_links_long.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_links_long.log; exit 1; }
      timeout -k 10 300 python3 -u tools/stress_paths.py --checksums --seconds 180 --seed 2031 > $OUT/stress_paths_long.log 2>&1 || { echo STRESS_FAIL; tail -5 $OUT/stress_paths_long.log; exit 1; }
      for f in stress_parity_long stress_fused_long stress_links_long stress_paths_long; do tail -1 $OUT/$f.log | cut -c1-200; done ;;
    repeat)
      timeout -k 10 400 python3 -u bench.py > $OUT/bench_default.log 2>&1 || { echo BENCH_FAIL; tail -20 $OUT/bench_default.log; exit 1; }
      tail -1 $OUT/bench_default.log | cut -c1-200
      for k in 1 2; do
        timeout -k 10 300 python3 -u tools/prof_checksums.py --no-device --paths 2000 --path-runs 6 > $OUT/validator_paths_$k.log 2>&1 || { echo VAL_FAIL; tail -20 $OUT/validator_paths_$k.log; exit 1; }
      done ;;
    valshapes)
      timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 20000 --path-kib 16 256 --path-runs 4 > $OUT/validator_small_files.log 2>&1 || { echo VALSHAPES_FAIL; tail -20 $OUT/validator_small_files.log; exit 1; }
      timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 150 --path-kib 16384 61440 --path-runs 4 > $OUT/validator_large_files.log 2>&1 || { echo VALSHAPES_FAIL; tail -20 $OUT/validator_large_files.log; exit 1; }
      timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 40 --path-kib 131072 196608 --path-runs 3 > $OUT/validator_streamed_files.log 2>&1 || { echo VALSHAPES_FAIL; tail -20 $OUT/validator_streamed_files.log; exit 1; }
      grep -h '"files"' $OUT/validator_*_files.log | cut -c1-300 ;;
    streamab)
      for k in 1 2; do
        for v in intree ${STREAM_VARIANTS:-stream_old}; do
          lib=""; [ $v != intree ] && lib=$R/tools/ablib/$v.so
          SD_HIP_CAS_LIB=$lib timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 40 --path-kib 131072 196608 --path-runs 4 > $OUT/streamed_${v}_$k.log 2>&1 || { echo STREAMAB_FAIL; tail -20 $OUT/streamed_${v}_$k.log; exit 1; }
          SD_HIP_CAS_LIB=$lib timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 1 --path-kib 4194304 4194305 --path-runs 4 > $OUT/onefile_${v}_$k.log 2>&1 || { echo STREAMAB_FAIL; tail -20 $OUT/onefile_${v}_$k.log; exit 1; }
        done
      done
      grep -h '"files"' $OUT/streamed_*.log $OUT/onefile_*.log | cut -c1-200 ;;
    smalltrace)
      SD_CAS_TRACE=1 timeout -k 10 400 python3 -u tools/prof_checksums.py --no-device --paths 20000 --path-kib 16 256 --path-runs 4 > $OUT/small_trace.log 2>&1 || { echo SMALLTRACE_FAIL; tail -20 $OUT/small_trace.log; exit 1; }
      grep sd_cas_trace $OUT/small_trace.log | grep "n=20000" | cut -c1-300 ;;
    suite)
      timeout -k 10 900 python3 -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1 || { echo PYTEST_FAIL; tail -30 $OUT/pytest_gpu.log; exit 1; }
      tail -1 $OUT/pytest_gpu.log ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo SESSION_OK
