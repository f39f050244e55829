#!/bin/bash
# Rebuild libgwaoi.so here (CPU); only if that succeeds, run the given gpurun command.
set -e
cd /root/repo
python -c "from goworld_amd import build; build.build(force=True)"
exec /usr/local/graft/bin/gpurun "$@"
