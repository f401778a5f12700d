# A/B of k_tcn shader cycles between this tree and another checkout (e.g. `git worktree add var/head HEAD`, built),
# alternating, R launches per run (tools/jitter.py).
# usage: bash tools/ab_tree.sh <tag> <rounds> <launches> <other-tree> [VAR=value for this tree]
set -o pipefail
tag=$1; rounds=$2; R=$3; other=$4; envs=${5:-}
out=$PWD/gpurun_out/$tag; mkdir -p $out
for r in $(seq 1 $rounds); do
  (cd $other && SEPVAD_TCN_CLOCK=1 timeout -k 10 120 python3 tools/jitter.py $R > $out/other.$r.txt 2>&1) || exit 1
  echo "other $r $(grep '^SUMMARY' $out/other.$r.txt)"
  env $envs SEPVAD_TCN_CLOCK=1 timeout -k 10 120 python3 tools/jitter.py $R > $out/this.$r.txt 2>&1 || exit 1
  echo "this $r $(grep '^SUMMARY' $out/this.$r.txt)"
done | tee $out/abt.txt
