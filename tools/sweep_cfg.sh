set -e
for c in 0 8 9 10 11 12 13 1 3; do
  echo "== cfg $c"
  KMAN_CHECK=0 KMAN_SORT_CFG=$c timeout -k 10 200 python tools/sortbench.py --reps 2 2>&1 | tail -1
done
