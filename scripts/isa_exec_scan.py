"""For every v_permlane*_swap in a kernel, walk back to the nearest instruction that writes EXEC
(s_and_saveexec / s_or_b64 exec / s_mov_b64 exec / s_andn2...) or a label, and print it."""
import re, sys
f, kern = sys.argv[1], sys.argv[2]
lines = open(f).read().split("\n")
s = next(i for i, l in enumerate(lines) if l.startswith(kern + ":"))
e = next(i for i in range(s, len(lines)) if "s_endpgm" in lines[i])
from collections import Counter
c = Counter()
for i in range(s, e):
    l = lines[i].split(";")[0].strip()
    if "permlane" in l and "swap" in l:
        j = i - 1
        while j > s:
            t = lines[j].split(";")[0].strip()
            if t.endswith(":"):
                c["label"] += 1; break
            if re.search(r"\bexec\b", t) and t.split()[0].startswith("s_"):
                c[t.split()[0] + " " + ("exec-dst" if t.split()[1].startswith("exec") else "saveexec")] += 1
                if "saveexec" in t or t.split()[1].startswith("exec"):
                    print(i + 1, "<-", j + 1, t)
                break
            j -= 1
print(c)
