#!/bin/bash
O=${GRAFT_REPO_ROOT:-$(pwd)}/gpurun_out/patchpmc; mkdir -p $O
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 90 rocprofv3 --pmc SQ_WAVES SQ_BUSY_CYCLES SQ_WAVE_CYCLES SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_WAIT_INST_ANY -d $O/p1 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/patch_probe.py $PE $PP > $O/p1.log 2>&1; echo rc $?
timeout -s KILL 90 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAIT_ANY SQ_INST_CYCLES_VMEM_RD GRBM_GUI_ACTIVE -d $O/p2 -o run --output-format csv -- python3 $GRAFT_REPO_ROOT/tools/patch_probe.py $PE $PP > $O/p2.log 2>&1; echo rc $?
