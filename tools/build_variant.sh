#!/bin/bash
# Build a measurement variant of the engine: variants/NAME/libbls381.so with extra hipcc flags.
#   bash tools/build_variant.sh NAME -DBLS_FE_WAVES_PER_EU=1 ...
set -e
cd "$(dirname "$0")/.."
NAME=$1; shift
python - "$NAME" "$@" <<'PY'
import os, sys
sys.path.insert(0, "consensus-specs_amd")
import build_native
name, flags = sys.argv[1], sys.argv[2:]
build_native.build_hip(force=True, extra=tuple(flags), out=os.path.join("variants", name, "libbls381.so"))
PY
