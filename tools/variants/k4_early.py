"""Ablation (timing only, wrong results): K4 (k_vit_chain_seg) returning after the barrier
list (phase A): the launch, the summary loads and the list alone."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "    // B. gap composites and windows, one lane per barrier."
assert old in s
s = s.replace(old, "    if (nbar >= 0) return;\n" + old, 1)
open(p, 'w').write(s)
