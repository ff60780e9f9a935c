# PMC passes over one GEMM case: 8ph (SCHED 1) and mmdx at 8192^3 fwd and dgrad
set -u
cd /tmp && export TMPDIR=/tmp && cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/pmcg
P1="SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE GRBM_GUI_ACTIVE"
P2="SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES GRBM_GUI_ACTIVE"
for c in "fwd 8192 8192 8192" "dgrad 8192 8192 8192"; do
  n=$(echo $c | cut -d' ' -f1)
  for arm in "" "--mmdx"; do
    t=${n}$(echo $arm | tr -d -)
    timeout -s KILL 90 rocprofv3 --pmc $P1 -d gpurun_out/pmcg/${t}_1 -o run --output-format csv -- python tools/gemm8ph_one.py $c $arm > gpurun_out/pmcg/${t}_1.log 2>&1 || { echo "fail $t 1"; exit 1; }
    timeout -s KILL 90 rocprofv3 --pmc $P2 -d gpurun_out/pmcg/${t}_2 -o run --output-format csv -- python tools/gemm8ph_one.py $c $arm > gpurun_out/pmcg/${t}_2.log 2>&1 || { echo "fail $t 2"; exit 1; }
    echo done $t
  done
done
