# ResNet-50 PMC passes (one counter set per run): MFMA busy, LDS conflicts, waits
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${1:-r3s2l_pmc_rn}
bash scripts/gpu_pmc.sh ${TAG}_1 "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VMEM_RD" --model resnet50 --steps 2 --warmup 1 --no-graph && \
bash scripts/gpu_pmc.sh ${TAG}_2 "SQ_WAIT_INST_LDS SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_MFMA SQ_INSTS_VMEM_WR SQ_WAVES GRBM_GUI_ACTIVE GRBM_COUNT" --model resnet50 --steps 2 --warmup 1 --no-graph && \
for t in 1 2; do python3 scripts/pmc_table.py $(find gpurun_out/${TAG}_$t/prof -name "*counter_collection.csv" | head -1) > gpurun_out/${TAG}_$t/pmc.txt; done && \
cut -c1-250 gpurun_out/${TAG}_1/pmc.txt | grep -E "kernel|igemm|bnh|head" && cut -c1-250 gpurun_out/${TAG}_2/pmc.txt | grep -E "kernel|igemm|bnh|head"
