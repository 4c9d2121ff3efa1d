# A/B: first-layer rows read from the precomputed table by the tiles (default) vs phase A's copy
# into the graph's table (MD_VARIANT bit 1)
for v in 0 1 0 1; do
  echo "MD_VARIANT=$v"
  MD_VARIANT=$v timeout -k 10 60 python scripts/spec_prof.py 2>&1 | head -1
  MD_VARIANT=$v timeout -k 10 60 python scripts/s0_prof.py
done
MD_VARIANT=0 timeout -k 10 60 python scripts/batch_prof.py 256 | grep "^batch"
