#!/usr/bin/env bash
# Builds reference-side checker binaries from /root/reference sources in place, outputs only
# into oracle/_ref/ (git-ignored, travels to the GPU box). Only the pcg32 demo compiles
# from the reference's own files without stand-in headers: every Nori translation unit
# includes include/nori/common.h -> <ImathPlatform.h> (IlmBase, absent) and the BVH /
# ImageBlock units need TBB headers (absent), so the renderer itself is unbuildable here.
set -euo pipefail
REF=${REFERENCE_ROOT:-/root/reference}
OUT="$(cd "$(dirname "$0")" && pwd)/_ref"
if [ ! -d "$REF/ext/pcg32" ]; then
  echo "build_ref: $REF not present, skipping" >&2
  exit 0
fi
mkdir -p "$OUT"
# pcg32.h uses std::iter_swap without including <algorithm> (Nori includes it first);
# -include supplies that standard header, no reference file is altered or stubbed.
g++ -O2 -std=c++11 -include algorithm -I"$REF/ext/pcg32" "$REF/ext/pcg32/pcg32-demo.cpp" -o "$OUT/pcg32-demo"
echo "built $OUT/pcg32-demo"
# Eigen evaluation-order probe (oracle/eigen_probe.cpp, test infrastructure) against the reference's
# vendored Eigen 3.3.8, x86-64 SSE2 without FMA contraction as the reference is built
if [ -d "$REF/ext/eigen/Eigen" ]; then
  g++ -O2 -std=c++17 -ffp-contract=off -I"$REF/ext/eigen" "$(dirname "$0")/eigen_probe.cpp" -o "$OUT/eigen_probe"
  echo "built $OUT/eigen_probe"
fi
# Transform probe (oracle/eigen_xform_probe.cpp, test infrastructure): the parser's transform composition,
# Matrix4f::inverse (SSE path) and the camera's sampleToCamera, evaluated by the reference's own Eigen
if [ -d "$REF/ext/eigen/Eigen" ]; then
  g++ -O2 -std=c++17 -ffp-contract=off -I"$REF/ext/eigen" "$(dirname "$0")/eigen_xform_probe.cpp" -o "$OUT/eigen_xform_probe"
  echo "built $OUT/eigen_xform_probe"
fi
# Texture / normal-map probe (oracle/normalmap_probe.cpp, test infrastructure): PNGTexture's decode loops, eval's
# normal-map blend, the mesh TBN product and the sphere re-framing, over the reference's own lodepng + Eigen 3.3.8.
# Built twice: with g++ and with clang++, whose argument evaluation orders differ (the "order" mode reports
# Point2f(nextFloat(), nextFloat()) as each compiler evaluates it).
if [ -d "$REF/ext/eigen/Eigen" ] && [ -f "$REF/ext/lodepng/src/lodepng.cpp" ]; then
  PROBE_FLAGS="-O2 -std=c++17 -ffp-contract=off -include algorithm -I$REF/ext/eigen -I$REF/ext/lodepng/include -I$REF/ext/pcg32"
  g++ $PROBE_FLAGS "$(dirname "$0")/normalmap_probe.cpp" "$REF/ext/lodepng/src/lodepng.cpp" -o "$OUT/normalmap_probe"
  echo "built $OUT/normalmap_probe"
  CLANGXX=/opt/rocm/llvm/bin/clang++
  if [ -x "$CLANGXX" ]; then
    "$CLANGXX" $PROBE_FLAGS "$(dirname "$0")/normalmap_probe.cpp" "$REF/ext/lodepng/src/lodepng.cpp" \
      -o "$OUT/normalmap_probe_clang"
    echo "built $OUT/normalmap_probe_clang"
  fi
fi
# Radiance .hdr probe (oracle/hdr_probe.cpp, test infrastructure): the reference's own HDRLoader.h, a self-contained
# header, on the test's synthetic files
if [ -f "$REF/include/nori/HDRLoader.h" ]; then
  g++ -O2 -std=c++17 -ffp-contract=off -I"$REF/include" "$(dirname "$0")/hdr_probe.cpp" -o "$OUT/hdr_probe"
  echo "built $OUT/hdr_probe"
fi
# The reference's statistical tests (oracle/hypothesis_probe.cpp, test infrastructure): ext/hypothesis/hypothesis.h
if [ -f "$REF/ext/hypothesis/hypothesis.h" ]; then
  g++ -O2 -std=c++17 -I"$REF/ext/hypothesis" "$(dirname "$0")/hypothesis_probe.cpp" -o "$OUT/hypothesis_probe"
  echo "built $OUT/hypothesis_probe"
fi
