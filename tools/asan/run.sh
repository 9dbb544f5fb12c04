#!/bin/bash
# AddressSanitizer build of the host side of the packer TUs (nrt_pack / nrt_common / nrt_prog:
# fragment layouts, index maps, weight programs) and a driver that packs every MLP shape the path
# uses (pack_driver.cpp).  ASan is applied to host code only (-Xarch_host); device code is compiled
# for gfx950 as usual but never launched: this runs on the CPU and stops at the first device
# allocation.  Output: build_asan/ (git-ignored).
set -euo pipefail
cd "$(dirname "$0")/../.."
OUT=build_asan
mkdir -p "$OUT"
HIPCC=${HIPCC:-/opt/rocm/bin/hipcc}
SAN=(-Xarch_host -fsanitize=address -Xarch_host -fno-omit-frame-pointer)
objs=()
for s in nrt_common.hip nrt_pack.hip nrt_prog.hip; do
  o="$OUT/${s%.hip}.o"
  "$HIPCC" --offload-arch=gfx950 -O1 -g -std=c++20 -fPIC "${SAN[@]}" -Iinclude \
    -Ineural_raytracing_amd/csrc -c "neural_raytracing_amd/csrc/$s" -o "$o" &
  objs+=("$o")
done
wait
"$HIPCC" --offload-host-only -O1 -g -std=c++20 "${SAN[@]}" -Iinclude -c tools/asan/pack_driver.cpp \
  -o "$OUT/pack_driver.o"
"$HIPCC" -fsanitize=address -fno-gpu-sanitize -o "$OUT/pack_driver" "$OUT/pack_driver.o" "${objs[@]}" \
  -L/opt/rocm/lib -lrocblas -Wl,-rpath,/opt/rocm/lib
ASAN_OPTIONS=detect_leaks=0 "$OUT/pack_driver"
