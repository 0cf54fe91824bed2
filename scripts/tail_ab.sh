set -e
for cfg in "128 64 20 125" "64 64 40 250" "32 64 80 500"; do
  for t in tail_check_old tail_check tail_check_old tail_check; do
    echo "== $t $cfg"; timeout -k 10 120 ./tools/$t $cfg 20 | grep -E "variant|shipped|<|hash|phases|max"
  done
done
