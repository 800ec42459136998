#!/usr/bin/env bash
# build the product library with extra HIP flags into optix-renderer_amd/NAME (A/B variants)
# usage: scripts/build_variant.sh NAME "-DFOO=1 ..."
set -eu
make -s -j8 OBJDIR=build/obj_$1 LIBDIR=optix-renderer_amd/$1 EXTRA_HIP="$2" optix-renderer_amd/$1/libnori_hip.so
