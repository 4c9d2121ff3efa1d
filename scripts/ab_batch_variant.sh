# A/B of one MD_VARIANT bit on the 256- and 512-graph batches (alternating, two rounds)
V=${1:-1}
for r in 1 2; do
  for v in 0 $V; do
    for nb in 256 512; do
      echo -n "MD_VARIANT=$v NB=$nb: "; MD_VARIANT=$v timeout -k 10 60 python scripts/batch_prof.py $nb | grep "^batch"
    done
  done
done
