#!/bin/bash
# Build A/B variants of the native extension into ab/NAME.so, then restore the default in-tree build:
#   tools/ab_build.sh FILES NAME1 "FLAGS1" [NAME2 "FLAGS2" ...]
# FILES: comma-separated csrc basenames the variant flags apply to (e.g. mlp_block5.hip); the other
# objects come from the shared object cache.  Compare with tools/so_ab.sh.
set -e
files=$1; shift
mkdir -p ab
SO=$(python -c "import sys; sys.path.insert(0,'.'); from dct_amd import _build; print(_build.target_path())")
while [ $# -gt 0 ]; do
  AB_HIPCC_FILES=$files AB_HIPCC_FLAGS="$2" python -c "import sys; sys.path.insert(0,'.'); from dct_amd import _build; _build.build()"
  cp "$SO" "ab/$1.so"; echo "ab/$1.so <- $2"
  shift 2
done
python -c "import sys; sys.path.insert(0,'.'); from dct_amd import _build; _build.build()"
