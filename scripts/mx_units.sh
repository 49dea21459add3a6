cd $GRAFT_REPO_ROOT
for u in 1 2 4 8 16 32; do
  echo "units/block $u"
  RSAC_MX_UNITS=$u timeout -k 10 60 python3 scripts/tune_score.py 32 2>&1 | grep variant
done
