#!/bin/bash
# Round 2: full GPU suite + smoke
set -o pipefail
cd "$GRAFT_REPO_ROOT"
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/r2i_pytest_gpu.log 2>&1
echo "pytest gpu exit=$?"
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r2i_smoke.log 2>&1
echo "smoke exit=$?"
