# r5l (closed-form 4D parser: tests, A/B, trace) then r5h (per-call PMC, zfp_parallel)
bash tools/sessions/r5l.sh || exit 1
bash tools/sessions/r5h.sh
