#!/usr/bin/env bash
# Drop-in for the reference's run script (code/run): same two arguments, same defaults,
# same result directories; the rollouts run on the MI355X through libmdroll.so.
#   ./run.sh MultiDismantler_unit_cost testSynthetic
#   ./run.sh MultiDismantler_degree_cost testReal
set -e
HERE="$(cd "$(dirname "$0")" && pwd)"
if [ $# -ge 2 ]; then
    address_dirtory=$1
    input_filename=$2
    shift 2
else
    address_dirtory='MultiDismantler_unit_cost'
    input_filename='train'
fi
case "$address_dirtory" in
    MultiDismantler_degree_cost) variant=degree; tag=degreecost ;;
    MultiDismantler_unit_cost)   variant=unit;   tag=unitcost ;;
    *) echo "No training or testing will be performed!"; exit 0 ;;
esac
case "$input_filename" in
    testReal)      out="../../results/$tag/MultiDismantler_real" ;;
    testSynthetic) out="../../results/$tag/MultiDismantler_syn/" ;;
    drawLmcc)      out="../../results/$tag/MultiDismantler_audc/" ;;
    *)             out="." ;;
esac
PYTHONPATH="$HERE${PYTHONPATH:+:$PYTHONPATH}" exec python -u -m mdcommunity_amd.cli "$variant" "$input_filename" --output "$out" "$@"
