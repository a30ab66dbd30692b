set -o pipefail
for s in "64 312 1000 30" "64 256 1000 30" "64 128 1000 30" "8 312 1000 30"; do
  LAM_ONLY_NEW=1 timeout -k 10 120 ./tools/lambench/lambench $s 50 || exit 1
done
