#!/bin/bash
# PMC breakdown of the coverage kernels (one counter group per pass; no tracing domains).
set -u
cd "$(dirname "$0")/.."
mkdir -p gpurun_out
export TMPDIR=/tmp
i=0
for grp in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" \
           "SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_INSTS_SALU SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_LDS SQ_LDS_BANK_CONFLICT GRBM_GUI_ACTIVE GRBM_COUNT" ; do
    i=$((i+1))
    rm -rf gpurun_out/pmc$i
    timeout -k 10 600 rocprofv3 --pmc $grp --output-format csv -d gpurun_out/pmc$i -o run -- python3 bench.py --steps 5 --warmup 1 --no-cpu > gpurun_out/pmc$i.log 2>&1
    rc=$?
    echo "pmc group $i rc=$rc"
    case $rc in 0|1) ;; *) exit $rc ;; esac
done
