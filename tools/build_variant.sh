#!/bin/bash
# Build a librm variant with extra -D flags for A/B timing (tools/ab_kernel.py).
#   tools/build_variant.sh NAME [-DFOO=1 ...]   -> tools/variants/librm_NAME.so
#   tools/build_variant.sh NAME --rev GITREV    -> librm built from a committed revision
#   tools/build_variant.sh NAME --patch F.diff  -> librm built with a patch applied
#   KOPT=-O3 tools/build_variant.sh NAME         -> the built-in kernels at another -O level
#                                                 (experiments live as patches, not knobs)
set -e
name=$1; shift
root=$(cd "$(dirname "$0")/.." && pwd)
out=$root/tools/variants; mkdir -p "$out"
src=$root
if [ "$1" = "--rev" ]; then
  src=$(mktemp -d); git -C "$root" archive "$2" | tar -x -C "$src"; shift 2
fi
if [ "$1" = "--patch" ]; then
  p=$(cd "$(dirname "$2")" && pwd)/$(basename "$2")
  if [ "$src" = "$root" ]; then src=$(mktemp -d); (cd "$root" && tar -c --exclude=.git --exclude=gpurun_out --exclude=tools/variants .) | tar -x -C "$src"; fi
  (cd "$src" && patch -s -p1 < "$p"); shift 2
fi
pkg=opengl-raymarching-in-compute-shader_amd
flags="--offload-arch=gfx950 -O3 -std=c++17 -fPIC -ffp-contract=off -fhip-fp32-correctly-rounded-divide-sqrt -I$src/include $*"
b=$(mktemp -d)
/opt/rocm/bin/hipcc $flags -c "$src/$pkg/csrc/rm_api.hip" -o "$b/rm_api.o" &
/opt/rocm/bin/hipcc $flags -fno-slp-vectorize -c "$src/$pkg/csrc/rm_table.hip" -o "$b/rm_table.o" &
# rm_kernels.hip as the Makefile builds it (both objects without SLP; RM_PIXEL_SLP=1
# builds k_pixel with it, the round-3 flags), except
# for the RM_STATS build, whose counters must live in one code object
case "$*" in
  *RM_STATS*) /opt/rocm/bin/hipcc $flags -c "$src/$pkg/csrc/rm_kernels.hip" -o "$b/rm_kernels.o" & ;;
  *) pslp=-fno-slp-vectorize; [ -n "$RM_PIXEL_SLP" ] && pslp=-fslp-vectorize
     /opt/rocm/bin/hipcc $flags ${KOPT:--O2} $pslp -DRM_KERNELS_PIXEL_ONLY -c "$src/$pkg/csrc/rm_kernels.hip" -o "$b/rm_kernels.o" &
     /opt/rocm/bin/hipcc $flags ${KOPT:--O2} -fno-slp-vectorize -DRM_KERNELS_AA_ONLY -c "$src/$pkg/csrc/rm_kernels.hip" -o "$b/rm_kernels_aa.o" & ;;
esac
/opt/rocm/bin/hipcc $flags -x c++ -c "$src/$pkg/csrc/rm_host.cpp" -o "$b/rm_host.o" &
[ -f "$src/$pkg/csrc/rm_comm.cpp" ] && { /opt/rocm/bin/hipcc $flags -x hip -c "$src/$pkg/csrc/rm_comm.cpp" -o "$b/rm_comm.o" & }
if [ -f "$src/$pkg/csrc/rm_jit.hip" ]; then  # per-table hiprtc kernels: embed the table sources
  c=$src/$pkg/csrc
  python3 "$src/$pkg/tools/embed_sources.py" "$b/rm_jit_src.inc" rm_table.hip=$c/rm_table.hip \
    rm_internal.hpp=$c/rm_internal.hpp rm_scene.hpp=$c/rm_scene.hpp rm_fastmath.hpp=$c/rm_fastmath.hpp \
    $( [ -f "$c/rm_shard.hpp" ] && echo rm_shard.hpp=$c/rm_shard.hpp ) \
    ../../include/rm_api.h=$src/include/rm_api.h
  /opt/rocm/bin/hipcc $flags -I"$b" -c "$c/rm_jit.hip" -o "$b/rm_jit.o" &
fi
for j in $(jobs -p); do wait "$j" || { echo "build_variant: a compile failed" >&2; exit 1; }; done
/opt/rocm/bin/hipcc --offload-arch=gfx950 -shared -fPIC -o "$out/librm_$name.so" "$b"/*.o -lhiprtc -ldl
rm -rf "$b"; [ "$src" != "$root" ] && rm -rf "$src"
echo "$out/librm_$name.so"
