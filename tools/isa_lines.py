"""Instructions of one kernel in a `hipcc --cuda-device-only -S -gline-tables-only` listing, grouped
by the source line (.loc) they are attributed to.  tools only (the gfx950 shape study).
  python tools/isa_lines.py LISTING.s KERNEL_SUBSTRING FILE_SUBSTRING LO HI [--dump]
prints the function's size, spill / scratch lines, and every instruction attributed to FILE lines
LO..HI (in listing order, with its line)."""
import re
import sys


def main():
    path, kname, fsub, lo, hi = sys.argv[1], sys.argv[2], sys.argv[3], int(sys.argv[4]), int(sys.argv[5])
    dump = "--dump" in sys.argv
    files = {}
    body, inside = [], False
    for line in open(path):
        m = re.match(r'\s*\.file\s+(\d+)\s+"([^"]*)"(?:\s+"([^"]*)")?', line)
        if m:
            files[int(m.group(1))] = (m.group(2) + "/" + (m.group(3) or "")).rstrip("/")
            continue
        if not inside and re.match(r"^" + r"\S*" + re.escape(kname) + r"\S*:", line):
            inside = True
        if inside:
            body.append(line.rstrip("\n"))
            if line.startswith(".Lfunc_end"):
                break
    cur, n, sel = None, 0, []
    for line in body:
        m = re.match(r"\s*\.loc\s+(\d+)\s+(\d+)", line)
        if m:
            cur = (int(m.group(1)), int(m.group(2)))
            continue
        s = line.strip()
        if not s or s.startswith((".", ";")) or s.endswith(":"):
            continue
        n += 1
        if cur and fsub in files.get(cur[0], "") and lo <= cur[1] <= hi:
            sel.append((cur[1], s))
    print("%s: %d instructions; %d attributed to %s:%d-%d" % (kname, n, len(sel), fsub, lo, hi))
    spills = sum(1 for ln in body if "Folded Spill" in ln)
    reloads = sum(1 for ln in body if "Folded Reload" in ln)
    print("  spill stores %d, reloads %d" % (spills, reloads))
    if dump:
        for l, s in sel:
            print("%5d  %s" % (l, s))


if __name__ == "__main__":
    main()
