#!/bin/bash
# closing check: full GPU suite (with the interaction's 16-B alignment contract) + smoke + bench
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/gpu_full.sh r03am
