# r5p (index scan with plausible starts) then r5o (look-back pre-pass A/B)
bash tools/sessions/r5p.sh || exit 1
bash tools/sessions/r5o.sh
