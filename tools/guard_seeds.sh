# loss-parity guard settings over several batches (tools/guard_seeds.py, one process per setting)
cd "${GRAFT_REPO_ROOT:-/root/repo}" && mkdir -p gpurun_out
SEEDS=${SEEDS:-0,1000,7,42,123}
for set in "dflt 7 4 10" "A 9 5 11" "B 8 5 11" "C 9 6 12"; do
  set -- $set
  KC=$2 TE=$3 TT=$4 timeout -k 10 400 python3 tools/guard_seeds.py $SEEDS $1 >> gpurun_out/guard_seeds.jsonl 2>> gpurun_out/guard_seeds.err || { echo "setting $1 failed"; exit 1; }
done
