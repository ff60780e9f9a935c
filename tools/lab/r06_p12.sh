# round 6: nontemporal stores of the BiLSTM forward's saved gates / cells and nontemporal
# gate loads in the backward (written once, read a step later) — C4 / C3 paired
set -o pipefail
R=$(pwd)
mkdir -p gpurun_out
run() { local label=$1 to=$2; shift 2; timeout -k 10 $to "$@" > $R/gpurun_out/$label.log 2>&1; local rc=$?; echo "[$label] rc=$rc"; [ $rc -le 1 ] || exit $rc; }
run p12_t 300 python -u -m pytest tests/test_text_gpu.py -x -q --timeout 120 --timeout-method thread -p no:cacheprovider -k lstm
for i in 1 2; do
  run p12_c4_def_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntlstm/libmmdx_hip.so run p12_c4_nt_$i 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline
  run p12_c3_def_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
  MMDX_LIB_PATH=$R/abtmp/ntlstm/libmmdx_hip.so run p12_c3_nt_$i 300 python bench.py --config c3 --steps 20 --warmup 5 --no-cpu-baseline
done
