#!/bin/bash
cd "${GRAFT_REPO_ROOT:-.}"
for V in ${VARIANTS:-fzref}; do
echo "--- $V"
mkdir -p /tmp/pkg$V && cp -r attack-vc_amd/*.py /tmp/pkg$V/ && cp scripts/dbg/$V/libavc.so /tmp/pkg$V/
AVC_PKG=/tmp/pkg$V timeout -k 10 200 python scripts/dbg/short_t.py || exit 1
done
