"""Print the NUMA node and local CPU list of HIP device 0 (PCI sysfs), and a CPU list on another node.

  python tools/numa_probe.py            -> "<node> <local cpulist> <remote cpulist>"
Used by tools/numa_ab.sh to pin the C2 probe next to / away from the GPU (host-memory mailbox round trips).
"""
import ctypes
import glob
import os


def bus_id(dev=0):
    hip = ctypes.CDLL("libamdhip64.so")
    buf = ctypes.create_string_buffer(64)
    if hip.hipDeviceGetPCIBusId(buf, 64, dev) != 0:
        raise RuntimeError("hipDeviceGetPCIBusId failed")
    return buf.value.decode().lower()


def read(path):
    with open(path) as f:
        return f.read().strip()


def main():
    bid = bus_id()
    dev = "/sys/bus/pci/devices/" + bid
    node = int(read(dev + "/numa_node"))
    local = read(dev + "/local_cpulist")
    remote = ""
    for n in sorted(glob.glob("/sys/devices/system/node/node*")):
        k = int(os.path.basename(n)[4:])
        if k != node:
            remote = read(n + "/cpulist")
            break
    print(node, local, remote or local)


if __name__ == "__main__":
    main()
