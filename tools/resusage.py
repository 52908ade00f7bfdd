"""Summarise hipcc -Rpass-analysis=kernel-resource-usage output (one line per kernel)."""
import re
import sys

text = open(sys.argv[1]).read().split("Function Name: ")[1:]
SCR = "ScratchSize \\[bytes/lane\\]"
for blk in text:
    name = blk.split()[0]

    def g(k):
        m = re.search(k + r": (\d+)", blk)
        return m.group(1) if m else "?"
    print("%-62s V%-4s scratch %-4s sgpr-spill %-4s vgpr-spill %s"
          % (name[:62], g("VGPRs"), g(SCR), g("SGPRs Spill"), g("VGPRs Spill")))
