# build libtt2 with csrc/decode_persist.hip replaced by $1 into $2 (A/B experiments; in-tree build untouched)
set -e
SRC=$1; OUT=$2
D=$(mktemp -d)
cp -r tacotron-2_amd/csrc $D/csrc && cp $SRC $D/csrc/decode_persist.hip && mkdir -p $D/include && cp include/tt2.h $D/include/
sed -i 's#../../include/tt2.h#../include/tt2.h#' $D/csrc/common.h
for f in gemm tacotron decode_persist wavenet griffinlim train step wavenet_wide train_front emt cbhg; do
  /opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Wno-unused-function -Wno-unused-variable -Wno-pass-failed -c $D/csrc/$f.hip -o $D/$f.o &
done
wait
/opt/rocm/bin/hipcc -shared --offload-arch=gfx950 -o $OUT $D/*.o -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
rm -rf $D
