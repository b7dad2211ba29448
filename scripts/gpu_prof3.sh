# PMC passes for one ablation mode of an alternative build.  usage: gpu_prof3.sh TAG DBG VARIANT [WORKLOAD]
TAG=${1:-p}; DBG=${2:-0}; V=${3:-new}; W=${4:-cfg2}
O=gpurun_out/$TAG
cd "$GRAFT_REPO_ROOT" && mkdir -p $O && export TMPDIR=/tmp && export AIRS_LIB=exp/$V/libairscmp.so && \
AIRS_DBG=$DBG timeout -k 10 300 rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_WAVE_CYCLES SQ_BUSY_CYCLES -d $O/p1 -o p1 -- python3 scripts/kbench.py $W > $O/p1.log 2>&1 && \
AIRS_DBG=$DBG timeout -k 10 300 rocprofv3 --pmc SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR GRBM_GUI_ACTIVE -d $O/p2 -o p2 -- python3 scripts/kbench.py $W > $O/p2.log 2>&1
