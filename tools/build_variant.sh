# builds lib_ab/libkc_NAME.so: the engine with extra compile flags for the counting kernels
# (A/B of compile-time knobs, loaded through KC_LIB).  usage: tools/build_variant.sh NAME "-DKNOB=V ..."
set -e
NAME=$1; FLAGS=$2
P=canonical-k-mer-hash-table_amd
B=lib_ab/build_$NAME
mkdir -p $B
HIPFLAGS="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -Wall -Wno-unused-result -Wno-unused-value $FLAGS"
for w in 1 2 3 4 5 6 7 8 9 10 11 12 13 14 15; do
  /opt/rocm/bin/hipcc $HIPFLAGS -DKC_W=$w -c $P/csrc/kc_count_w.hip -o $B/kc_count_w$w.o &
  if (( w % 8 == 0 )); then wait; fi
done
wait
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -o lib_ab/libkc_$NAME.so $P/build/kc_tokenize.o $P/build/kc_util.o \
    $P/build/kc_count.o $P/build/kc_skm.o $B/kc_count_w*.o $P/build/kc_compact_w*.o $P/build/kc_api.o -lpthread
echo lib_ab/libkc_$NAME.so
