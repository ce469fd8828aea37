"""Where the host process runs relative to the GPU: the CPUs it may use, the GPU's
PCI-local CPUs (sysfs), and config B's step time (host-bound at 100k Gaussians)
unpinned and pinned to the allowed CPUs local to the GPU.
usage (on the box): python tools/numa_probe.py"""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "3dgs_study_amd"), ROOT]

import torch  # noqa: E402

import synthetic  # noqa: E402
import train_step  # noqa: E402


def cpulist(s):
    out = set()
    for part in s.strip().split(","):
        if "-" in part:
            a, b = part.split("-")
            out.update(range(int(a), int(b) + 1))
        elif part:
            out.add(int(part))
    return out


def main():
    allowed = sorted(os.sched_getaffinity(0))
    print("allowed cpus", len(allowed), allowed[:8], "...", flush=True)
    p = torch.cuda.get_device_properties(0)
    bus = getattr(p, "pci_bus_id", None)
    dom = getattr(p, "pci_domain_id", 0)
    dev_id = getattr(p, "pci_device_id", None)
    print("pci", dom, bus, dev_id, flush=True)
    local = set()
    if bus is not None:
        bdf = f"{dom:04x}:{bus:02x}:{dev_id:02x}.0" if dev_id is not None else None
        for path in (f"/sys/bus/pci/devices/{bdf}/local_cpulist", f"/sys/bus/pci/devices/{bdf}/numa_node"):
            try:
                print(path, open(path).read().strip(), flush=True)
            except OSError as e:
                print(path, "unreadable", e, flush=True)
        try:
            local = cpulist(open(f"/sys/bus/pci/devices/{bdf}/local_cpulist").read())
        except OSError:
            pass
    both = sorted(set(allowed) & local)
    print("allowed & local", len(both), both[:16], flush=True)
    dev = torch.device("cuda:0")
    cfg = synthetic.CONFIGS["B"]
    cam = synthetic.make_camera(cfg["W"], cfg["H"], view=0).to(dev)
    g = synthetic.make_gaussians(cfg["P"], cfg["sh_degree"], seed=0).to(dev, requires_grad=True)
    target = synthetic.make_target(cfg["W"], cfg["H"], seed=1).to(dev)
    bg = torch.zeros(3, device=dev)
    params = g.params()

    def step():
        for q in params:
            q.grad = None
        train_step.train_step(cam, g, target, bg, glue="fused")

    def rate(n=300):
        for _ in range(30):
            step()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            step()
        torch.cuda.synchronize()
        return 1e3 * (time.perf_counter() - t0) / n

    for r in range(3):
        os.sched_setaffinity(0, allowed)
        a = rate()
        b = None
        if both:
            os.sched_setaffinity(0, both)
            b = rate()
        c = None
        os.sched_setaffinity(0, [allowed[0]])
        c = rate()
        print(f"round {r}: unpinned {a:.4f} ms  local {b if b is None else round(b, 4)} ms  one cpu {c:.4f} ms",
              flush=True)


if __name__ == "__main__":
    main()
