#!/bin/bash
# PMC passes (FETCH_SIZE, WRITE_SIZE; one rocprofv3 run each) over the c4, c5 and c3 legs.
cd "${GRAFT_REPO_ROOT:-/root/repo}"
set -e
LEG=c4 FAMILY=k_mv_expand,k_mv_apply,k_mv_small,k_mv_gather MARKER=k_mv_gather ROUNDS=5,24 bash scripts/r03_pmc_legs.sh
LEG=c5 FAMILY=k_mv_expand,k_mv_apply,k_mv_small,k_mv_gather MARKER=k_mv_gather ROUNDS=3,12 PMC_TO=600 bash scripts/r03_pmc_legs.sh
LEG=c3 FAMILY=k_bin_small,k_bin_expand,k_bin_apply,k_bin_gather,k_bin_seed MARKER=k_bin_gather ALL=1 bash scripts/r03_pmc_legs.sh
