"""Ablation (timing only, wrong results): K4 (k_vit_chain_seg) without its serial chain over the
barriers — the staged windows are still built, the chain walk is skipped."""
import sys
p = sys.argv[1]
s = open(p).read()
old = "    const bool all_staged = nst == nbar && sWoff[nst] <= kStageSteps;\n    if (all_staged) {"
assert old in s
s = s.replace(old, "    const bool all_staged = nst == nbar && sWoff[nst] <= kStageSteps;\n    if (false) {")
s = s.replace("    } else if (t < 64) {\n        double2 v = init;\n        for (int i = 0; i < nbar; ++i) {",
              "    } else if (false) {\n        double2 v = init;\n        for (int i = 0; i < nbar; ++i) {")
open(p, 'w').write(s)
