#!/bin/bash
# round 6 final: the full GPU suite + smoke() + the default bench (scripts/gpu_default.sh), then rocprofv3 profiles
# of the training lines at HEAD (TAG r06f)
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
bash scripts/gpu_default.sh || exit $?
TAG=${TAG:-r06f} LINES="train_step train_step_refcfg" bash scripts/gpu_profiles.sh
