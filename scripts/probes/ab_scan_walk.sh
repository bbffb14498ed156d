#!/bin/bash
# Round 2: GPU tests with the queue cut walk in production, an interleaved A/B of the production
# scan against sweep variants 31 (round-2 walk: min over the 8 summary slots per cut) and 29 (plain
# rolling state), then the round-end profile (smoke, rocprofv3 stats, PMC passes) and the bench.
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}" || exit 1
bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread" \
  "ab:300:CONFIGS='prod:;walk8:SDFS_SCAN_VARIANT=31;plain:SDFS_SCAN_VARIANT=29' ROUNDS=12 python scripts/ab.py" \
  "ab4k:300:CONFIGS='prod:;walk8:SDFS_SCAN_VARIANT=31' ROUNDS=8 MIN_SEG_KIB=2 MASK_BITS=11 python scripts/ab.py" \
  "bench:240:python bench.py" || exit $?
bash scripts/final_profile.sh
