import gc, sys, time, runpy
stats = {0: [0, 0.0], 1: [0, 0.0], 2: [0, 0.0]}
t = {}
def cb(phase, info):
    g = info["generation"]
    if phase == "start":
        t[g] = time.perf_counter()
    else:
        stats[g][0] += 1
        stats[g][1] += time.perf_counter() - t[g]
gc.callbacks.append(cb)
sys.argv = ["bench.py", "--steps", "20", "--warmup", "3"]
try:
    runpy.run_path("bench.py", run_name="__main__")
finally:
    print("gc:", {g: (n, round(s * 1e3, 2)) for g, (n, s) in stats.items()}, file=sys.stderr)
