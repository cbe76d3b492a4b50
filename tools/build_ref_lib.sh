# builds lib_ab/libkc_NAME.so from the sources of a git ref (the A/B base of a working-tree change).
# usage: tools/build_ref_lib.sh NAME [REF]
set -e
NAME=$1; REF=${2:-HEAD}
T=$(mktemp -d)
git archive $REF canonical-k-mer-hash-table_amd/csrc include | tar -x -C $T
mkdir -p lib_ab
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value"
H=/opt/rocm/bin/hipcc
S=$T/canonical-k-mer-hash-table_amd/csrc
B=$T/build; mkdir -p $B
$H $HIPFLAGS -c $S/kc_tokenize.hip -o $B/kc_tokenize.o &
$H $HIPFLAGS -c $S/kc_util.hip -o $B/kc_util.o &
$H $HIPFLAGS -c $S/kc_count.hip -o $B/kc_count.o &
[ -f $S/kc_skm.hip ] && $H $HIPFLAGS -c $S/kc_skm.hip -o $B/kc_skm.o &
$H $HIPFLAGS -x hip -c $S/kc_api.cpp -o $B/kc_api.o &
wait
for w in 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15; do
  $H $HIPFLAGS -DKC_W=$w -c $S/kc_count_w.hip -o $B/kc_count_w$w.o &
  $H $HIPFLAGS -DKC_W=$w -c $S/kc_compact_w.hip -o $B/kc_compact_w$w.o &
  if (( w % 4 == 0 )); then wait; fi
done
wait
$H --offload-arch=gfx950 -shared -o lib_ab/libkc_$NAME.so $B/*.o -lpthread
rm -rf $T
echo lib_ab/libkc_$NAME.so
