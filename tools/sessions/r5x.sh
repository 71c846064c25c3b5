# r5z (suite, smoke, bench lines, kernel trace) then r5y (per-call PMC of C3 and C5)
bash tools/sessions/r5z.sh || exit 1
bash tools/sessions/r5y.sh
