"""Turn a rocprofv3 kernel_stats.csv into a markdown table (top-N kernels)."""
import csv
import sys


def main(path, top=25, per=1):
    rows = list(csv.DictReader(open(path)))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"Total GPU kernel time: {tot / 1e6:.2f} ms" + (f" ({tot / 1e6 / per:.2f} ms per unit of {per})" if per > 1 else ""))
    print()
    print("| % | total ms | calls | avg us | kernel |")
    print("|---:|---:|---:|---:|---|")
    for r in rows[:top]:
        name = r["Name"].replace("|", "/")
        if len(name) > 100:
            name = name[:100] + "..."
        print(f"| {float(r['Percentage']):.1f} | {float(r['TotalDurationNs']) / 1e6:.2f} | {r['Calls']} | "
              f"{float(r['AverageNs']) / 1e3:.1f} | `{name}` |")


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 25, int(sys.argv[3]) if len(sys.argv) > 3 else 1)
