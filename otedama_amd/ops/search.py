"""Python-facing launchers for the gfx950 search kernels on torch-owned buffers.

These are the "ops" of the framework: each call enqueues a HIP kernel on the
current torch stream (so it composes with RCCL collectives issued through
``torch.distributed`` on the same device) and returns immediately; results are
read back with :meth:`SearchResult.nonces` after a synchronize.

Kernels (csrc/kernels):
  * ``otd_sha256d_search``   — SHA-256d nonce search (K1)
  * ``otd_sha256d_search_k`` — K version variants per lane sharing the block-2 schedule
  * ``otd_sha256d_search_v`` / ``_vn<NC>`` — 64 x NC version variants per wave (NC per lane), block-2 schedule on
    the scalar unit
  * ``otd_scrypt_*``         — scrypt N=1024,r=1,p=1 three-stage search (K5)
  * ``x11k::k_*512_*``       — X11 eleven-stage chain, one kernel per stage (K6)
"""
from __future__ import annotations

from dataclasses import dataclass

import torch

from otedama_amd.ops.native import require_native

from otedama_amd.ops.tuning import (  # noqa: F401  (re-exported: launch geometry lives in the torch-free module)
    SCRYPT_BLOCKS_PER_CU,
    SHA256D_BLOCKS_PER_CU,
    SHA256D_K_BLOCKS_PER_CU,
    SHA256D_V2_BLOCKS_PER_CU,
    SHA256D_V_BLOCKS_PER_CU,
)


def _device_index(device) -> int:
    d = torch.device(device)
    return 0 if d.index is None else d.index


def default_grid(device, blocks_per_cu: int) -> int:
    n = require_native()
    cus = n.gpu_cu_count(_device_index(device)) or 256
    return cus * blocks_per_cu


@dataclass
class SearchResult:
    buf: torch.Tensor  # int32 [1 + cap]: count, nonces
    cap: int

    def count(self) -> int:
        return int(self.buf[0].item()) & 0xFFFFFFFF

    def nonces(self) -> list[int]:
        host = self.buf.cpu().tolist()
        n = min(host[0] & 0xFFFFFFFF, self.cap)
        return [x & 0xFFFFFFFF for x in host[1 : 1 + n]]


class Sha256dSearch:
    """Reusable SHA-256d search launcher bound to one device."""

    def __init__(self, device="cuda:0", cap: int = 1024, grid: int | None = None):
        self.native = require_native()
        self.device = torch.device(device)
        self.cap = cap
        self.grid = grid or default_grid(self.device, SHA256D_BLOCKS_PER_CU)
        self.out = torch.zeros(1 + cap, dtype=torch.int32, device=self.device)

    def prepare(self, header80: bytes, target32: bytes) -> bytes:
        return self.native.sha256d_prepare(header80, target32)

    def launch(self, params: bytes, base: int = 0, count: int = 1 << 32, out: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> SearchResult:
        out = self.out if out is None else out
        if out.numel() < 1 + self.cap or out.dtype != torch.int32 or out.device != self.device:
            raise ValueError("out must be an int32 tensor of >= 1+cap elements on the search device")
        stream = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):  # the count reset must precede the kernel on the launch stream
            out[:1].zero_()
        self.native.launch_sha256d(params, base & 0xFFFFFFFF, int(count), out.data_ptr(), self.cap, self.grid,
                                   stream.cuda_stream)
        return SearchResult(out, self.cap)

    def search(self, header80: bytes, target32: bytes, base: int = 0, count: int = 1 << 32) -> list[int]:
        r = self.launch(self.prepare(header80, target32), base, count)
        torch.cuda.synchronize(self.device)
        return r.nonces()


@dataclass
class SearchResultK:
    buf: torch.Tensor  # int32 [1 + 2*cap]: count, (nonce, variant) pairs
    cap: int

    def count(self) -> int:
        return int(self.buf[0].item()) & 0xFFFFFFFF

    def hits(self) -> list[tuple[int, int]]:
        host = self.buf.cpu().tolist()
        n = min(host[0] & 0xFFFFFFFF, self.cap)
        return [(host[1 + 2 * i] & 0xFFFFFFFF, host[2 + 2 * i]) for i in range(n)]


class Sha256dSearchK:
    """SHA-256d over K header variants at once (BIP320 version rolling): the variants share block 2 of the
    first hash (bytes 64..79), so each lane computes that message schedule once for K midstates."""

    def __init__(self, device="cuda:0", k: int = 4, cap: int = 1024, grid: int | None = None):
        self.native = require_native()
        if k not in self.native.SHA256D_K_VALUES:
            raise ValueError(f"k must be one of {self.native.SHA256D_K_VALUES}")
        self.k = k
        self.device = torch.device(device)
        self.cap = cap
        self.grid = grid or default_grid(self.device, SHA256D_K_BLOCKS_PER_CU)
        self.out = torch.zeros(1 + 2 * cap, dtype=torch.int32, device=self.device)

    def prepare(self, headers: list[bytes], target32: bytes) -> bytes:
        if len(headers) != self.k:
            raise ValueError(f"need exactly {self.k} headers")
        return self.native.sha256d_prepare_k(list(headers), target32)

    def launch(self, params: bytes, base: int = 0, count: int = 1 << 32, out: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> SearchResultK:
        out = self.out if out is None else out
        if out.numel() < 1 + 2 * self.cap or out.dtype != torch.int32 or out.device != self.device:
            raise ValueError("out must be an int32 tensor of >= 1+2*cap elements on the search device")
        stream = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):  # the count reset must precede the kernel on the launch stream
            out[:1].zero_()
        self.native.launch_sha256d_k(params, base & 0xFFFFFFFF, int(count), out.data_ptr(), self.cap, self.grid,
                                     stream.cuda_stream)
        return SearchResultK(out, self.cap)

    def search(self, headers: list[bytes], target32: bytes, base: int = 0, count: int = 1 << 32) -> list[tuple[int, int]]:
        r = self.launch(self.prepare(headers, target32), base, count)
        torch.cuda.synchronize(self.device)
        return r.hits()


@dataclass
class PreparedV:
    params: bytes         # Sha256dParamsV (kernarg)
    vars: torch.Tensor    # uint8 device copy of the Sha256dVariant table (72 B per variant)
    n: int                # variants (multiple of 64)


class Sha256dSearchV:
    """Version-parallel SHA-256d (csrc/kernels/sha256d_search_v.hip): the 64 lanes of a wave are 64 header
    variants with identical bytes 64..79 and the wave walks W3 (the big-endian nonce word) together, so the
    first hash's message schedule runs on the scalar unit. Hits are (nonce, variant index) pairs; a launch over
    W3 in [base, base + count) covers the nonces bswap(W3) of that range for every variant."""

    def __init__(self, device="cuda:0", cap: int = 1024, grid: int | None = None, occupancy8: bool = True,
                 block: int = 256, chains: int = 1):
        """chains=2..4: that many variants per lane on the same nonce (64 x chains per wave); with chains=2
        ``occupancy8`` selects the 5-waves/SIMD build instead of the 4-wave one."""
        self.native = require_native()
        if chains not in (1, 2, 3, 4):
            raise ValueError("chains must be 1..4")
        self.chains = chains
        self.group = self.native.SHA256D_V_GROUP * chains
        self.occupancy8 = occupancy8
        if block not in (64, 256):
            raise ValueError("block must be 64 or 256 threads")
        self.block = block
        self.device = torch.device(device)
        self.cap = cap
        self.grid = grid or default_grid(self.device, SHA256D_V_BLOCKS_PER_CU)
        self.out = torch.zeros(1 + 2 * cap, dtype=torch.int32, device=self.device)

    def prepare(self, headers: list[bytes], target32: bytes) -> PreparedV:
        if not headers or len(headers) % self.group:
            raise ValueError(f"need a positive multiple of {self.group} headers")
        groups = len(headers) // self.group
        waves = self.grid * self.block // 64
        if waves % groups:
            raise ValueError(f"the wave count ({waves}) must be a multiple of the variant groups ({groups})")
        params, table = self.native.sha256d_prepare_v(list(headers), target32)
        vars_dev = torch.frombuffer(bytearray(table), dtype=torch.uint8).to(self.device)
        return PreparedV(params, vars_dev, len(headers))

    def launch(self, prep: PreparedV, base: int = 0, count: int = 1 << 32, out: torch.Tensor | None = None,
               stream: torch.cuda.Stream | None = None) -> SearchResultK:
        out = self.out if out is None else out
        if out.numel() < 1 + 2 * self.cap or out.dtype != torch.int32 or out.device != self.device:
            raise ValueError("out must be an int32 tensor of >= 1+2*cap elements on the search device")
        if prep.vars.device != self.device:
            raise ValueError("variant table must live on the search device")
        if prep.vars.numel() != prep.n * 72 or len(prep.params) != self.native.SHA256D_V_PARAMS_SIZE:
            raise ValueError("prepared table does not match its parameter block")
        cur = torch.cuda.current_stream(self.device)
        if stream is None:
            stream = cur
        elif stream != cur:
            stream.wait_stream(cur)  # prepare() uploaded the variant table on the current stream
        with torch.cuda.stream(stream):
            out[:1].zero_()
        self.launch_into(prep, base, count, out, stream)
        return SearchResultK(out, self.cap)

    def launch_into(self, prep: PreparedV, base: int, count: int, out: torch.Tensor, stream) -> None:
        """Append this range's hits to ``out`` on ``stream``, with no zeroing and no stream ordering: for pipelined
        callers that zero ``out`` once and spread one window over several launches on alternating streams (hit
        slots are claimed atomically, so concurrent launches may share one buffer)."""
        self.native.launch_sha256d_v(prep.params, prep.vars.data_ptr(), base & 0xFFFFFFFF, int(count),
                                     out.data_ptr(), self.cap, self.grid, stream.cuda_stream, self.occupancy8,
                                     self.block, self.chains)

    def search(self, headers: list[bytes], target32: bytes, base: int = 0, count: int = 1 << 32) -> list[tuple[int, int]]:
        r = self.launch(self.prepare(headers, target32), base, count)
        torch.cuda.synchronize(self.device)
        return r.hits()


class ScryptSearch:
    """scrypt(1024,1,1) search: PBKDF2-in -> ROMix (HBM scratchpad) -> PBKDF2-out."""

    def __init__(self, device="cuda:0", cap: int = 1024, grid: int | None = None, gap: int = 1,
                 lanes_per_slot: int = 1, kernel: str = "coop"):
        """kernel="coop": lane-cooperative full-line ROMix (gap 1 only, the fast path);
        kernel="coop2": the same with two software-pipelined hashes per lane;
        kernel="split": the cooperative ROMix as two launches (pad writes, then lookups), one hash per lane slot;
        kernel="lane": one lane per hash with lookup gap 1/2/4. Raw native codes
        (SCRYPT_COOP / SCRYPT_COOP2 / SCRYPT_COOP_SPLIT / SCRYPT_LANE_W8) may also be passed as ``gap``."""
        self.native = require_native()
        codes = {"coop": self.native.SCRYPT_COOP, "coop2": self.native.SCRYPT_COOP2,
                 "split": self.native.SCRYPT_COOP_SPLIT}
        if kernel not in ("coop", "coop2", "split", "lane"):
            raise ValueError(f"kernel must be 'coop', 'coop2', 'split' or 'lane', got {kernel!r}")
        if kernel in codes and gap == 1:
            gap = codes[kernel]
        self.kernel = {v: k for k, v in codes.items()}.get(gap, "lane")
        if self.kernel == "split" and lanes_per_slot != 1:
            raise ValueError("the split kernel holds one hash per lane slot")
        self.device = torch.device(device)
        self.cap = cap
        self.gap = gap
        self.grid = grid or default_grid(self.device, SCRYPT_BLOCKS_PER_CU // (2 if self.kernel == "coop2" else 1))
        self.batch = self.grid * 256 * lanes_per_slot * (2 if self.kernel == "coop2" else 1)
        nbytes = self.native.scrypt_scratch_bytes(self.grid, gap)
        self.scratch = torch.empty(nbytes, dtype=torch.uint8, device=self.device)
        self.xbuf = torch.empty(self.batch * 128, dtype=torch.uint8, device=self.device)
        self.out = torch.zeros(1 + cap, dtype=torch.int32, device=self.device)

    @property
    def scratch_bytes(self) -> int:
        return self.scratch.numel()

    def prepare(self, header80: bytes, target32: bytes) -> bytes:
        return self.native.scrypt_prepare(header80, target32)

    def launch(self, params: bytes, base: int = 0, count: int | None = None,
               stream: torch.cuda.Stream | None = None) -> SearchResult:
        count = self.batch if count is None else count
        if not 0 < count <= self.batch:
            raise ValueError(f"count must be in [1, {self.batch}]")
        stream = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):
            self.out[:1].zero_()
        self.native.launch_scrypt(params, base & 0xFFFFFFFF, int(count), self.xbuf.data_ptr(),
                                  self.scratch.data_ptr(), self.gap, self.out.data_ptr(), self.cap, self.grid,
                                  stream.cuda_stream)
        return SearchResult(self.out, self.cap)

    def search(self, header80: bytes, target32: bytes, base: int = 0, count: int | None = None) -> list[int]:
        r = self.launch(self.prepare(header80, target32), base, count)
        torch.cuda.synchronize(self.device)
        return r.nonces()


X11_BATCH = 1 << 23  # nonces per chain launch: 512 MiB of 64-byte digests, ~20-40 ms of work


class X11Search:
    """X11 search: eleven stage kernels over a 64 B/nonce digest buffer (8 u64 planes),
    the target compare fused into the ECHO stage. ``trace`` runs the chain stage by
    stage and returns every intermediate digest (for the per-stage numerics tests)."""

    def __init__(self, device="cuda:0", cap: int = 1024, batch: int = X11_BATCH):
        self.native = require_native()
        self.device = torch.device(device)
        self.cap = cap
        self.batch = int(batch)
        if not 0 < self.batch <= 1 << 26:
            raise ValueError("batch must be in [1, 2^26]")
        self.H = torch.empty(8 * self.batch, dtype=torch.int64, device=self.device)
        self.out = torch.zeros(1 + cap, dtype=torch.int32, device=self.device)

    def prepare(self, header80: bytes, target32: bytes) -> bytes:
        return self.native.x11_prepare(header80, target32)

    def launch(self, params: bytes, base: int = 0, count: int | None = None,
               stream: torch.cuda.Stream | None = None) -> SearchResult:
        count = self.batch if count is None else count
        if not 0 < count <= self.batch:
            raise ValueError(f"count must be in [1, {self.batch}]")
        stream = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(stream):
            self.out[:1].zero_()
        self.native.launch_x11(params, base & 0xFFFFFFFF, self.H.data_ptr(), self.batch, int(count),
                               self.out.data_ptr(), self.cap, stream.cuda_stream)
        return SearchResult(self.out, self.cap)

    def search(self, header80: bytes, target32: bytes, base: int = 0, count: int | None = None) -> list[int]:
        r = self.launch(self.prepare(header80, target32), base, count)
        torch.cuda.synchronize(self.device)
        return r.nonces()

    def trace(self, header80: bytes, base: int, count: int) -> list[torch.Tensor]:
        """Digests after each of the 11 stages: list of uint8 [count, 64] CPU tensors."""
        if not 0 < count <= self.batch:
            raise ValueError(f"count must be in [1, {self.batch}]")
        params = self.prepare(header80, bytes(32))
        stream = torch.cuda.current_stream(self.device)
        planes = self.H.view(8, self.batch)
        out = []
        for st in range(self.native.X11_STAGES):
            self.native.launch_x11_stage(params, st, base & 0xFFFFFFFF, self.H.data_ptr(), self.batch, int(count),
                                         0, 0, stream.cuda_stream)
            torch.cuda.synchronize(self.device)
            words = planes[:, :count].t().contiguous().cpu()          # [count, 8] int64 (LE words)
            out.append(words.view(torch.uint8).reshape(count, 64))
        return out
