# A/B of MD_VARIANT values on the single-graph rollout (kernel ms per rollout, alternating)
for r in 1 2; do
  for v in 0 ${@:-1}; do
    echo -n "MD_VARIANT=$v: "; MD_VARIANT=$v timeout -k 10 60 python scripts/spec_prof.py 2>&1 | grep -E "^gmm|prebuild" | tr '\n' ' '; echo
  done
done
