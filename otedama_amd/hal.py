"""Hardware abstraction: device identities, capabilities, drivers, detection.

Parity: internal/hal/{device,registry,gpu_linux}.go
  * Family (asic|gpu|cpu), Identity(+validate), Capabilities ...... device.go:50-148
  * Device / Driver / Detector contracts ........................... device.go:155-217
  * Registry (sorted drivers, duplicate guard) ..................... registry.go:25-105
  * Detect: every driver in parallel, identity validation,
    partial-failure tolerant ....................................... registry.go:138-201
  * GPULinuxDriver: /sys/class/drm/renderD* presence detection,
    vendor 0x1002 = AMD, id "gpu-renderD128" ....................... gpu_linux.go:61-189

MI355X-native difference: the reference hard-codes ``SHA256d = False`` for
every GPU (gpu_linux.go:131) because it has no GPU compute. Here the HIP driver
enumerates devices through the native runtime and reports the kernels that
exist for the device's ISA: gfx950 -> sha256d, scrypt and x11. The DRM
driver is kept for non-HIP render nodes (presence only, no hashing), and
render nodes that the HIP driver already owns are not reported twice.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from dataclasses import dataclass, field
from enum import Enum
from typing import Callable, Protocol


class Family(str, Enum):
    ASIC = "asic"
    GPU = "gpu"
    CPU = "cpu"


class HalError(ValueError):
    pass


@dataclass(frozen=True)
class Identity:
    id: str
    family: Family
    vendor: str = ""
    model: str = ""

    def __str__(self) -> str:
        return f"{self.family.value}[{self.id}: {self.model or 'unknown'}]"

    def validate(self) -> None:
        if not self.id:
            raise HalError("hal: Identity.ID must not be empty")
        if not isinstance(self.family, Family):
            raise HalError(f"hal: Identity.Family {self.family!r} is not a valid Family")
        for ch in self.id:
            if ch in " \t\n/":
                raise HalError(f"hal: Identity.ID contains forbidden character {ch!r}")


@dataclass(frozen=True)
class Capabilities:
    sha256d: bool = False
    general_compute: bool = False
    scrypt: bool = False
    x11: bool = False

    def supports(self, algorithm: str) -> bool:
        return bool(getattr(self, algorithm, False))


class Device(Protocol):
    def identity(self) -> Identity: ...

    def capabilities(self) -> Capabilities: ...

    def shutdown(self) -> None: ...


@dataclass
class SimpleDevice:
    ident: Identity
    caps: Capabilities
    index: int = -1                 # HIP ordinal for GPUs
    threads: int = 0                # CPU threads
    extra: dict = field(default_factory=dict)

    def identity(self) -> Identity:
        return self.ident

    def capabilities(self) -> Capabilities:
        return self.caps

    def shutdown(self) -> None:
        return None


class Driver(Protocol):
    def name(self) -> str: ...

    def enumerate(self) -> list: ...


class CPUDriver:
    """The built-in CPU device (engine/setup.go:274-297): SHA256d + general compute."""

    def __init__(self, threads: int = 0):
        self.threads = threads or (os.cpu_count() or 1)

    def name(self) -> str:
        return "cpu"

    def enumerate(self) -> list:
        model = _cpu_model()
        # SHA-256d through the SHA-NI scanner; scrypt / X11 through the host reference chains (slow, CPU-only hosts)
        return [SimpleDevice(Identity("cpu-0", Family.CPU, _cpu_vendor(), model),
                             Capabilities(sha256d=True, general_compute=True, scrypt=True, x11=True),
                             threads=self.threads)]


# ISA -> kernels compiled into the native extension (csrc/kernels)
KERNEL_ISAS = {"gfx950": Capabilities(sha256d=True, general_compute=True, scrypt=True, x11=True)}


class HIPDriver:
    """GPU devices visible to the HIP runtime (one per ordinal)."""

    def __init__(self, native_loader: Callable | None = None):
        self._loader = native_loader

    def name(self) -> str:
        return "hip"

    def enumerate(self) -> list:
        try:
            if self._loader is not None:
                n = self._loader()
            else:
                from otedama_amd.ops.native import load

                n = load(build_if_missing=False)
        except Exception:  # noqa: BLE001
            return []
        if n is None:
            return []
        out = []
        for i in range(n.gpu_device_count()):
            arch = n.gpu_arch_name(i).split(":")[0]
            caps = KERNEL_ISAS.get(arch, Capabilities(general_compute=True))
            cus = n.gpu_cu_count(i)
            model = "AMD Instinct MI355X" if arch == "gfx950" else f"AMD GPU ({arch})"
            out.append(SimpleDevice(Identity(f"gpu-{i}", Family.GPU, "AMD", f"{model} {cus}CU {arch}"), caps,
                                    index=i, extra={"arch": arch, "cus": cus}))
        return out


KFD_TOPOLOGY_PATH = "/sys/class/kfd/kfd/topology/nodes"


def _kfd_props(path: str) -> dict[str, int]:
    out = {}
    for line in _read(path).splitlines():
        k, _, v = line.partition(" ")
        try:
            out[k] = int(v)
        except ValueError:
            pass
    return out


def _visible(n: int) -> list[int]:
    """HIP ordinals after HIP_VISIBLE_DEVICES / ROCR_VISIBLE_DEVICES / CUDA_VISIBLE_DEVICES (integer lists)."""
    idx = list(range(n))
    for var in ("ROCR_VISIBLE_DEVICES", "HIP_VISIBLE_DEVICES", "CUDA_VISIBLE_DEVICES"):
        v = os.environ.get(var)
        if v is None:
            continue
        sel = [int(x) for x in v.split(",") if x.strip().lstrip("-").isdigit()]
        idx = [idx[i] for i in sel if 0 <= i < len(idx)] if v.strip() else []
    return idx


class KFDDriver:
    """GPU devices from the KFD topology in sysfs, in HIP ordinal order, WITHOUT initialising a HIP runtime.

    Used when every device runs in its own process (engine/devproc.py): the engine process never opens the GPU,
    so the devices it hands out can only be named here and are opened by their own processes."""

    def __init__(self, base_path: str | None = None, dri_path: str = "/dev/dri"):
        self.base_path = base_path or KFD_TOPOLOGY_PATH
        self.dri_path = dri_path

    def name(self) -> str:
        return "hip"

    def _openable(self, props: dict[str, int]) -> bool:
        """The ROCm runtime skips a GPU node whose render device this process cannot open (a container given
        some of the host's GPUs still sees every node in the topology): the HIP ordinal space counts only the
        openable ones, so the list here must too, or ordinal i would name another GPU."""
        minor = props.get("drm_render_minor", -1)
        if minor is None or minor <= 0:
            return True  # an old kernel without the property: nothing to check against
        return os.access(os.path.join(self.dri_path, f"renderD{minor}"), os.R_OK | os.W_OK)

    def enumerate(self) -> list:
        try:
            nodes = sorted((int(d) for d in os.listdir(self.base_path) if d.isdigit()))
        except OSError:
            nodes = []
        if not nodes and self.base_path == KFD_TOPOLOGY_PATH and os.path.exists("/dev/kfd"):
            return HIPDriver().enumerate()  # sysfs topology not readable here: ask the runtime after all
        gpus = []
        for n in nodes:
            p = _kfd_props(os.path.join(self.base_path, str(n), "properties"))
            if p.get("simd_count", 0) <= 0 or not p.get("gfx_target_version"):
                continue  # a CPU node
            if not self._openable(p):
                continue  # not ours: the runtime will not count it either
            v = p["gfx_target_version"]
            arch = f"gfx{v // 10000}{(v // 100) % 100:x}{v % 100:x}"
            cus = p["simd_count"] // max(p.get("simd_per_cu", 4), 1)
            gpus.append((arch, cus))
        out = []
        for i, k in enumerate(_visible(len(gpus))):
            arch, cus = gpus[k]
            caps = KERNEL_ISAS.get(arch, Capabilities(general_compute=True))
            model = "AMD Instinct MI355X" if arch == "gfx950" else f"AMD GPU ({arch})"
            out.append(SimpleDevice(Identity(f"gpu-{i}", Family.GPU, "AMD", f"{model} {cus}CU {arch}"), caps,
                                    index=i, extra={"arch": arch, "cus": cus, "source": "kfd"}))
        return out


IOLINK_TYPES = {2: "pcie", 11: "xgmi"}  # hsakmttypes.h HSA_IOLINK_TYPE_PCIEXPRESS / HSA_IOLINK_TYPE_XGMI


def kfd_topology(base_path: str | None = None) -> dict:
    """The GPU-to-GPU links of the visible GPUs from the KFD topology (no HIP runtime): per GPU its HIP ordinal,
    KFD node, XGMI hive id and XGMI-optimised SDMA engines; per directed GPU pair the io_link's type (``xgmi`` /
    ``pcie`` / the raw number), weight and max bandwidth (MB/s, as KFD reports it). bench.py's comm section puts it
    beside the measured bus bandwidth, so an 8-GPU figure reads against the links it ran on. Empty off a ROCm host."""
    base = base_path or KFD_TOPOLOGY_PATH
    drv = KFDDriver(base)
    try:
        nodes = sorted(int(d) for d in os.listdir(base) if d.isdigit())
    except OSError:
        return {"gpus": [], "links": []}
    gpu_nodes = []
    props_of = {}
    for n in nodes:
        p = _kfd_props(os.path.join(base, str(n), "properties"))
        if p.get("simd_count", 0) > 0 and p.get("gfx_target_version") and drv._openable(p):
            gpu_nodes.append(n)
            props_of[n] = p
    order = [gpu_nodes[k] for k in _visible(len(gpu_nodes))]
    index_of = {n: i for i, n in enumerate(order)}
    gpus = [{"index": i, "node": n, "hive_id": props_of[n].get("hive_id"),
             "sdma_xgmi_engines": props_of[n].get("num_sdma_xgmi_engines")} for i, n in enumerate(order)]
    links = []
    for n in order:
        ldir = os.path.join(base, str(n), "io_links")
        try:
            entries = sorted(os.listdir(ldir), key=lambda x: int(x) if x.isdigit() else 0)
        except OSError:
            continue
        for e in entries:
            lp = _kfd_props(os.path.join(ldir, e, "properties"))
            to = lp.get("node_to")
            if to not in index_of or to == n:
                continue
            t = lp.get("type", 0)
            links.append({"from": index_of[n], "to": index_of[to], "type": IOLINK_TYPES.get(t, t),
                          "weight": lp.get("weight"), "max_bandwidth": lp.get("max_bandwidth")})
    return {"gpus": gpus, "links": links}


DRM_BASE_PATH = "/sys/class/drm"


def infer_vendor_name(vendor_id: str) -> str:
    return {"0x10de": "NVIDIA", "0x1002": "AMD", "0x8086": "Intel"}.get(vendor_id.strip(), "Unknown GPU vendor")


def _read(path: str) -> str:
    try:
        with open(path) as f:
            return f.read().strip()
    except OSError:
        return ""


class GPULinuxDriver:
    """Presence-only render-node detection (gpu_linux.go). Capability: general compute only."""

    def __init__(self, base_path: str | None = None, skip_vendors: tuple[str, ...] = ()):
        self.base_path = base_path or DRM_BASE_PATH
        self.skip_vendors = skip_vendors

    def name(self) -> str:
        return "gpu_linux"

    def enumerate(self) -> list:
        try:
            entries = sorted(os.listdir(self.base_path))
        except OSError:
            return []
        seen, out = set(), []
        for name in entries:
            if not name.startswith("renderD"):
                continue
            dev_path = os.path.join(self.base_path, name, "device")
            canonical = os.path.realpath(dev_path)
            if canonical in seen:
                continue
            seen.add(canonical)
            vendor_id = _read(os.path.join(canonical, "vendor"))
            # Unreadable vendor = a node this process cannot use (e.g. another GPU's partition exposed in
            # a container's sysfs): reporting it would hand arbitration phantom devices.
            if not vendor_id or vendor_id in self.skip_vendors:
                continue
            vendor = infer_vendor_name(vendor_id)
            model = vendor + " GPU"
            for line in _read(os.path.join(canonical, "uevent")).splitlines():
                if line.startswith("PCI_ID="):
                    model = f"{vendor} GPU ({line[7:]})"
            ident = Identity(f"gpu-{name}", Family.GPU, vendor, model)
            try:
                ident.validate()
            except HalError:
                continue
            out.append(SimpleDevice(ident, Capabilities(sha256d=False, general_compute=True)))
        return out


class Registry:
    def __init__(self) -> None:
        self._lock = threading.Lock()
        self._drivers: dict[str, object] = {}

    def register(self, d) -> None:
        if d is None:
            raise HalError("hal: cannot register nil driver")
        name = d.name()
        if not name:
            raise HalError("hal: driver must have a non-empty name")
        with self._lock:
            if name in self._drivers:
                raise HalError(f"hal: driver {name!r} is already registered")
            self._drivers[name] = d

    def drivers(self) -> list:
        with self._lock:
            return [self._drivers[k] for k in sorted(self._drivers)]

    def lookup(self, name: str):
        with self._lock:
            return self._drivers.get(name)

    def __len__(self) -> int:
        return len(self._drivers)


class Detector:
    def __init__(self, registry: Registry | None = None, logger: Callable[[str, str, Exception], None] | None = None,
                 timeout: float = 30.0):
        self.registry = registry or Registry()
        self.logger = logger
        self.timeout = timeout

    def detect(self) -> list:
        """Enumerate every driver concurrently (registry.go:138-201). A driver that fails is logged and skipped;
        one that is still running after ``timeout`` is logged and abandoned (its daemon thread is not joined),
        and the devices of the drivers that finished are returned."""
        drivers = self.registry.drivers()
        if not drivers:
            return []
        results: queue.Queue = queue.Queue()

        def run(d):
            try:
                results.put((d, d.enumerate(), None))
            except Exception as exc:  # noqa: BLE001 - partial failure tolerated
                results.put((d, None, exc))

        for d in drivers:
            threading.Thread(target=run, args=(d,), name=f"otedama-hal-{d.name()}", daemon=True).start()
        out, pending = [], {d.name() for d in drivers}
        deadline = time.monotonic() + self.timeout
        while pending:
            try:
                d, devs, exc = results.get(timeout=max(0.0, deadline - time.monotonic()))
            except queue.Empty:
                for name in sorted(pending):
                    if self.logger:
                        self.logger(name, "enumerate timed out", TimeoutError(f"no result after {self.timeout} s"))
                break
            pending.discard(d.name())
            if exc is not None:
                if self.logger:
                    self.logger(d.name(), "enumerate failed", exc)
                continue
            for dev in devs or []:
                try:
                    dev.identity().validate()
                except HalError as exc:
                    if self.logger:
                        self.logger(d.name(), "device rejected due to invalid identity", exc)
                    continue
                out.append(dev)
        out.sort(key=lambda d: d.identity().id)
        return out


def default_registry(cpu_threads: int = 0, include_drm: bool = True, gpu_free: bool = False) -> Registry:
    """``gpu_free``: enumerate GPUs from the KFD topology instead of the HIP runtime (the process stays GPU-free;
    its devices run in device processes)."""
    r = Registry()
    r.register(CPUDriver(cpu_threads))
    r.register(KFDDriver() if gpu_free else HIPDriver())
    if include_drm:
        r.register(GPULinuxDriver(skip_vendors=("0x1002",)))  # AMD GPUs come from the HIP driver
    return r


def _cpu_model() -> str:
    for line in _read("/proc/cpuinfo").splitlines():
        if line.startswith("model name"):
            return line.split(":", 1)[1].strip()
    import platform

    return platform.processor() or "CPU"


def _cpu_vendor() -> str:
    for line in _read("/proc/cpuinfo").splitlines():
        if line.startswith("vendor_id"):
            return line.split(":", 1)[1].strip()
    return ""
