#!/bin/bash
# tp_fwd variants: parity (TP / model tests) + kbench timing each
set -e -o pipefail
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
cd "$R"
bash tools/ab_variants.sh main "$@"
