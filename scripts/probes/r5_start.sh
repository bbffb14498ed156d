cd $GRAFT_REPO_ROOT && bash scripts/gpu_session.sh \
  "gputests:600:python -u -m pytest tests -m gpu -x -q --timeout 150 --timeout-method thread" \
  "smoke:180:python -c 'import __graft_entry__ as g; g.smoke()'" \
  "bench:240:python bench.py" \
  "fforms:300:bash scripts/probes/fused_forms_r5.sh"
