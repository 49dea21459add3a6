set -e
for pp in 2 1 16; do echo "PP=$pp"; RSAC_SMALL_PP=$pp timeout -k 10 120 python scripts/prof_ms_to_best.py 2>&1 | grep device; done
