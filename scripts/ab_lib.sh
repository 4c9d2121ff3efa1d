# A/B of two builds on one box: MD_LIB=<alt .so> vs the in-tree libmdroll.so, alternating.
set -e
ALT=${1:-mdcommunity_amd/libmdroll_ab.so}
NB=${2:-256}
for r in 1 2; do
  echo "in-tree:"; timeout -k 10 60 python scripts/batch_prof.py $NB | grep "^batch"
  echo "alt ($ALT):"; MD_LIB=$ALT timeout -k 10 60 python scripts/batch_prof.py $NB | grep "^batch"
done
