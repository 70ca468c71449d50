#!/bin/bash
# TEST INFRASTRUCTURE ONLY: compiles the part of the reference's hot path that
# builds on its own -- the element operations of reduce-op.c (:71-150) -- from
# the source where it lies, into oracle/_ref/libref_ops.so.  It stays in this
# container: git-ignored, and listed in .gpurunignore so that neither the
# reference's text nor an object built from it ever reaches the GPU box (the
# GPU tests read tests/golden/ref_element_ops.json, the outputs it computed).
#
# The text is read between two markers and piped straight into gcc after
# <complex.h>, followed by oracle/ref_ops_harness.c (the exported wrapper);
# nothing of the reference is written to disk.  Flags are the reference's own
# defaults for gcc: -std=c99 -Wall with no -O (configure:523-528, 690-696),
# plus -fPIC -shared for a loadable object.
#
# Usage: oracle/build_ref.sh [REFERENCE_ROOT]   (default /root/reference)
set -euo pipefail
HERE="$(cd "$(dirname "$0")" && pwd)"
REF="${1:-/root/reference}"
SRC="$REF/src/reduce/reduce-op.c"
OUT="$HERE/_ref/libref_ops.so"

if [ ! -f "$SRC" ]; then
    echo "build_ref.sh: $SRC not present; oracle/_ref not built" >&2
    exit 0
fi

BEGIN='^#define SHMEM_MATH_FUNC'
END='^SHMEM_MINIMAX_FUNC (longdouble, long double);'
first=$(grep -n "$BEGIN" "$SRC" | cut -d: -f1)
last=$(grep -n "$END" "$SRC" | cut -d: -f1)
if [ -z "$first" ] || [ -z "$last" ] || [ "$first" -ne 71 ] || [ "$last" -ne 150 ]; then
    echo "build_ref.sh: element-op section of $SRC is not at :71-150 (found ${first:-?}-${last:-?})" >&2
    exit 1
fi

mkdir -p "$HERE/_ref"
[ "$OUT" -nt "$SRC" ] && [ "$OUT" -nt "$HERE/ref_ops_harness.c" ] && [ "$OUT" -nt "$0" ] && exit 0
{
    printf '#include <complex.h>\n#line %d "%s"\n' "$first" "$SRC"
    sed -n "${first},${last}p" "$SRC"
    cat "$HERE/ref_ops_harness.c"
} | gcc -std=c99 -Wall -fPIC -shared -x c - -o "$OUT.tmp"
mv "$OUT.tmp" "$OUT"
