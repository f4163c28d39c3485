"""Symbolize tools/sprof samples: python tools/sprof/report.py /tmp/sprof.out [top] [--inline] [--lines]
Prints the share of samples per function (the innermost inlined frame with --inline; with --lines
per outermost function and the innermost frame's source line)."""
import collections
import subprocess
import sys


def main(path, top=40, inline=False, by_line=False):
    maps, samples = [], []
    for line in open(path):
        if line.startswith("M "):
            parts = line[2:].split()
            if len(parts) >= 6 and "x" in parts[1]:
                lo, hi = (int(v, 16) for v in parts[0].split("-"))
                maps.append((lo, hi, int(parts[2], 16), parts[5]))
        elif line.startswith("S "):
            samples.append(int(line[2:], 16))
    by_obj = collections.defaultdict(list)
    for pc in samples:
        for lo, hi, off, obj in maps:
            if lo <= pc < hi:
                by_obj[obj].append(pc - lo + off)
                break
        else:
            by_obj["?"].append(pc)
    counts = collections.Counter()
    for obj, pcs in by_obj.items():
        if obj == "?" or not obj.startswith("/"):
            counts[obj] += len(pcs)
            continue
        uniq = sorted(set(pcs))
        args = ["addr2line", "-C", "-f", "-e", obj] + (["-i"] if inline else [])
        out = subprocess.run(args, input="\n".join("%x" % p for p in uniq), capture_output=True, text=True).stdout
        lines = out.splitlines()
        names = {}
        if by_line:
            for p in uniq:
                r = subprocess.run(["addr2line", "-C", "-f", "-i", "-e", obj, "%x" % p], capture_output=True, text=True)
                fr = r.stdout.splitlines()
                # frames innermost first: (function, file:line) pairs
                names[p] = ("%s | %s" % (fr[-2][:80], fr[1].split("/")[-1])) if len(fr) >= 2 else "?"
        elif inline:
            # with -i each address prints 2 lines per frame; take the first (innermost) frame
            i = 0
            res = subprocess.run(["addr2line", "-C", "-f", "-i", "-e", obj], input="\n".join("%x" % p for p in uniq),
                                 capture_output=True, text=True).stdout
            # fall back: one query per address (slow but exact)
            for p in uniq:
                r = subprocess.run(["addr2line", "-C", "-f", "-i", "-e", obj, "%x" % p], capture_output=True, text=True)
                fr = r.stdout.splitlines()
                names[p] = (fr[0] + " @ " + fr[1].split("/")[-1]) if fr else "?"
        else:
            for i, p in enumerate(uniq):
                names[p] = lines[2 * i] if 2 * i < len(lines) else "?"
        short = obj.split("/")[-1]
        for p in pcs:
            counts["%s: %s" % (short, names[p][:150])] += 1
    total = sum(counts.values())
    print("%d samples" % total)
    for name, c in counts.most_common(top):
        print("%6.2f%%  %s" % (100.0 * c / total, name))


if __name__ == "__main__":
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    main(args[0], int(args[1]) if len(args) > 1 else 40, "--inline" in sys.argv, "--lines" in sys.argv)
