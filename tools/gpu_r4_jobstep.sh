#!/bin/bash
# Round 4: the 100-file job step (tools/prof_jobstep.py) traced: host phases (SD_CAS_TRACE)
# and a rocprofv3 kernel + memory-copy trace.  Usage: gpu_r4_jobstep.sh <tag>
set -o pipefail
R=$GRAFT_REPO_ROOT
OUT=$R/gpurun_out/${1:-r4_jobstep}
mkdir -p $OUT
cd $R
SD_CAS_TRACE=1 timeout -k 5 120 python3 tools/prof_jobstep.py > $OUT/jobstep.log 2> $OUT/jobstep_trace.txt || { echo JOBSTEP_FAIL; tail -5 $OUT/jobstep.log; exit 1; }
cat $OUT/jobstep.log
cd /tmp && export TMPDIR=/tmp
timeout -k 5 200 rocprofv3 --kernel-trace --memory-copy-trace --stats -d $OUT/prof -o js --output-format csv -- python3 $R/tools/prof_jobstep.py > $OUT/jobstep_prof.log 2>&1 || { echo PROF_FAIL; tail -5 $OUT/jobstep_prof.log; exit 1; }
echo JOBSTEP_OK
