# tiles per queue item (MD_VARIANT bits 9-10 = tpi, 0 = default 2) x admission limit (bits 16+), 256 and 512 graphs
set -e
for T in 1 2 3; do
  for K in 64 96 128 160; do
    v=$(( (T << 9) + (K << 16) ))
    for NB in 256 512; do
      echo -n "tpi=$T K=$K NB=$NB: "; MD_VARIANT=$v timeout -k 10 60 python scripts/batch_prof.py $NB | grep "^batch"
    done
  done
done
