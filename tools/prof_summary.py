"""Summarise a rocprofv3 ``*_kernel_stats.csv`` into a markdown table (for profiles/)."""
import csv
import sys


def main(path, title=None, top=30):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    out = [f"## {title or path}", "", f"total kernel time {tot / 1e6:.2f} ms", "",
           "| % | calls | avg us | min us | max us | kernel |", "|---:|---:|---:|---:|---:|---|"]
    for r in rows[:top]:
        out.append(f"| {float(r['TotalDurationNs']) / tot * 100:.1f} | {r['Calls']} | "
                   f"{float(r['AverageNs']) / 1e3:.2f} | {float(r['MinNs']) / 1e3:.2f} | {float(r['MaxNs']) / 1e3:.2f} | "
                   f"`{r['Name'][:120]}` |")
    return "\n".join(out) + "\n"


if __name__ == "__main__":
    print(main(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else None))
