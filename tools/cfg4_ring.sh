#!/bin/bash
# cfg4's p pass against its r pass at several yk-ring depths (KRY_CG_YDEFER):
# a kernel trace per depth (tools/prof_cfg.sh cfg4 40), output
# gpurun_out/prof_cfg4_D<depth>/.
cd "$GRAFT_REPO_ROOT" || exit 1
for d in "$@"; do
  KRY_CG_YDEFER=$d PROF_TAG=D$d bash tools/prof_cfg.sh cfg4 40 || exit $?
done
