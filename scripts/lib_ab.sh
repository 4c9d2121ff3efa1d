#!/bin/bash
# A/B of the in-tree library against another build (MD_LIB), alternating processes:
#   [AB_MODES=k] bash scripts/lib_ab.sh OUTDIR OTHER_LIB GRAPHS [REPS]   (MD_DF=k, default 1)
O=$1; B=$2; G=$3; N=${4:-15}
mkdir -p $O
for r in 1 2; do
  for lib in "" "$B"; do
    tag=${lib:-intree}; tag=$(basename $tag)
    MD_LIB=${lib:+$PWD/$lib} timeout -k 10 300 env AB_MODES=${AB_MODES:-1} python -u scripts/df_ab.py $G $N > $O/ab_${tag}_$r.out 2> $O/ab_${tag}_$r.err || exit 1
    echo "== $tag pass $r"; cat $O/ab_${tag}_$r.out
  done
done
