# r6x: LDS bank conflicts and LDS-array busy of the headline kernels (never measured before)
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/pmc_pass.sh lds_cornell "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" && \
bash tools/pmc_pass.sh lds_blob "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES GRBM_GUI_ACTIVE" --preset config3
echo "r6x rc=$?"
