#!/bin/bash
# Build an alternative native library into variants/<name>.so with extra hipcc flags (A/B and
# timing experiments), then restore the default in-tree build.  Usage: tools/build_variant.sh <name> <flags...>
set -e
name=$1; shift
mkdir -p variants
FEDMI_HIPCC_FLAGS="$*" python -c "from fedmi.ops import build as b; import shutil; shutil.copy(b.build(force=True), 'variants/$name.so')"
python -c "from fedmi.ops import build as b; b.build(force=True)"
