# builds lib_ab/libkc_NAME.so with extra compile flags for EVERY translation unit (knobs that the
# host sizing shares with the kernels, e.g. KC_RUNW1).  usage: tools/build_variant_full.sh NAME "-DKNOB=V ..."
set -e
NAME=$1; FLAGS=$2
P=canonical-k-mer-hash-table_amd
B=lib_ab/build_$NAME
mkdir -p $B
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value $FLAGS"
H=/opt/rocm/bin/hipcc
$H $HIPFLAGS -c $P/csrc/kc_tokenize.hip -o $B/kc_tokenize.o &
$H $HIPFLAGS -c $P/csrc/kc_util.hip -o $B/kc_util.o &
$H $HIPFLAGS -c $P/csrc/kc_count.hip -o $B/kc_count.o &
$H $HIPFLAGS -c $P/csrc/kc_skm.hip -o $B/kc_skm.o &
$H $HIPFLAGS -x hip -c $P/csrc/kc_api.cpp -o $B/kc_api.o &
wait
for w in 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15; do
  $H $HIPFLAGS -DKC_W=$w -c $P/csrc/kc_count_w.hip -o $B/kc_count_w$w.o &
  $H $HIPFLAGS -DKC_W=$w -c $P/csrc/kc_compact_w.hip -o $B/kc_compact_w$w.o &
  if (( w % 4 == 0 )); then wait; fi
done
wait
$H --offload-arch=gfx950 -shared -o lib_ab/libkc_$NAME.so $B/*.o -lpthread
echo lib_ab/libkc_$NAME.so
