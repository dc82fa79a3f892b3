#!/bin/bash
# Build a kernel-variant library for A/B runs:
#   tools/build_variant.sh <name> <file.hip> <product object it replaces, e.g. attention> [hipcc flags]
# links build/*.o with <file.hip> in place of build/<object>.o -> build_ab/<name>.so
set -e
cd "$(dirname "$0")/../sam-quantization_amd"
name=$1; src=$2; base=$3; shift 3
mkdir -p build_ab
/opt/rocm/bin/hipcc -O3 -std=c++17 -fPIC --offload-arch=gfx950 -Icsrc "$@" -c "$src" -o "build_ab/$name.o"
/opt/rocm/bin/hipcc -shared -fPIC --offload-arch=gfx950 -o "build_ab/$name.so" $(ls build/*.o | grep -v "/$base.o") "build_ab/$name.o"
echo "build_ab/$name.so"
