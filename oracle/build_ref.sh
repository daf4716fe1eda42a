#!/usr/bin/env bash
# TEST INFRASTRUCTURE ONLY.
#
# Builds the REFERENCE arithmetic of the RS coding path -- ISA-L 2.22.0's
# pure-C erasure_code (ec_base.c + ec_base_aliases.c), exactly what
# /root/reference links via ncloud_code (src/common/CMakeLists.txt:5-8) --
# straight from the tarball vendored in the reference
# (third-party/isa-l-2.22.0.tar.gz, pinned at cmake/ExternalProjects.cmake:2-14).
#
# * Sources are extracted to a private temp dir and deleted afterwards; only
#   the built library lands in oracle/_ref/ (git-ignored, travels to the GPU
#   box as a prebuilt .so).  Nothing from the reference is copied into the repo.
# * ISA-L's SIMD .asm cannot be assembled here (no nasm/yasm); the base C
#   path is bit-identical by construction (ISA-L's erasure_code_test.c checks
#   SIMD against base).
# * rs.cc itself is NOT built: it needs glog, boost and the reference's
#   Config/Chunk headers, none of which exist in this image, so it is
#   "unbuildable here"; its glue logic is restated in nxec_oracle.c and
#   gen_golden.c (each citing rs.cc line numbers).
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
TARBALL="${NXEC_REF_TARBALL:-/root/reference/third-party/isa-l-2.22.0.tar.gz}"
OUT="$HERE/_ref"
if [ ! -f "$TARBALL" ]; then
  echo "build_ref: reference tarball not present ($TARBALL); skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
TMP="$(mktemp -d)"
trap 'rm -rf "$TMP"' EXIT
tar xzf "$TARBALL" -C "$TMP" \
  isa-l-2.22.0/erasure_code/ec_base.c isa-l-2.22.0/erasure_code/ec_base.h \
  isa-l-2.22.0/erasure_code/ec_base_aliases.c isa-l-2.22.0/include/erasure_code.h \
  isa-l-2.22.0/include/gf_vect_mul.h isa-l-2.22.0/include/types.h
SRC="$TMP/isa-l-2.22.0"
gcc -O2 -fPIC -shared -I"$SRC/include" -I"$SRC/erasure_code" \
  "$SRC/erasure_code/ec_base.c" "$SRC/erasure_code/ec_base_aliases.c" -o "$OUT/libisal_base.so"
# the generator links the reference library; its header is the public ISA-L API,
# declared locally in gen_golden.c (prototypes only)
gcc -O2 -std=c11 -Wall -o "$OUT/gen_golden" "$HERE/gen_golden.c" \
  -L"$OUT" -lisal_base -Wl,-rpath,'$ORIGIN' -lcrypto -lpthread
echo "build_ref: built $OUT/libisal_base.so and $OUT/gen_golden"
