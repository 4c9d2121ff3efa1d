# A/B of MD_VARIANT values on one box (same build), alternating: bash scripts/ab_variant.sh "0 512" 256
set -e
VS=${1:-"0 512"}
NB=${2:-256}
for r in 1 2; do
  for v in $VS; do
    echo -n "MD_VARIANT=$v: "; MD_VARIANT=$v timeout -k 10 60 python scripts/batch_prof.py $NB | grep "^batch"
  done
done
