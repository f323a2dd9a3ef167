"""Baseline-JPEG ingest on the device (csrc/jpeg.hip): torchvision.io.read_image(path, RGB) of
detect.py:55-58 split into a host entropy decode (one image per host thread; ctypes releases the GIL)
and a device reconstruction (dequantisation, islow IDCT, fancy upsampling, YCbCr -> RGB) that writes
the uint8 [B,3,H,W] batch the detector plans read, byte-identical to libjpeg's default decode.

    pk = packet(open(path, "rb").read())      # host: np.uint8 packet, or None if unsupported
    dec = BatchDecoder(device)
    dec.decode([pk0, pk1, ...], out_u8)        # device: out_u8 [B,3,H,W] uint8 (cuda tensor)

JPEGs the device path does not handle (progressive, arithmetic-coded, CMYK / RGB JPEGs, unusual
chroma samplings) come back as None from packet(); the caller decodes those files on the host.
"""
import ctypes

import numpy as np
import torch

from . import ops


class Packets(list):
    """The packets of one batch of equal-size images (a run_batches input: decoded on the device
    straight into the plan's uint8 input)."""

    def __init__(self, packets, hw):
        super().__init__(packets)
        self.hw = tuple(hw)


def packet(data, pinned=False):
    """Entropy-decode one JPEG file's bytes -> (packet, (H, W)); (None, reason) when the device path
    does not handle the file; raises EdgeDetError on corrupt data.  The packet is an np.uint8 array,
    or with pinned=True a pinned torch uint8 tensor (from torch's caching host allocator, so a
    batch's packets upload without a staging copy)."""
    L = ops.lib()
    buf = np.frombuffer(data, dtype=np.uint8)
    hw = (ctypes.c_int32 * 2)()
    # one decode into a buffer of a generous guess; a second only when the guess is too small
    cap = max(4096, 8 * buf.size + 65536)

    def alloc(k):
        if pinned:
            t = torch.empty(k, dtype=torch.uint8, pin_memory=True)
            return t, t.data_ptr()
        a = np.empty(k, np.uint8)
        return a, a.ctypes.data

    out, ptr = alloc(cap)
    n = L.edgedet_jpeg_packet(buf.ctypes.data, buf.size, ptr, cap, hw)
    if n == 0:
        return None, L.edgedet_last_error().decode()
    if n < 0:
        ops.check(int(n))
    if n > cap:
        out, ptr = alloc(int(n))
        m = L.edgedet_jpeg_packet(buf.ctypes.data, buf.size, ptr, int(n), hw)
        if m != n:
            ops.check(int(m) if m < 0 else -1)
    return out[:int(n)], (int(hw[0]), int(hw[1]))


class PackedBatch:
    """One batch of equal-size JPEG files entropy-decoded by edgedet_jpeg_batch_packets into a single
    pinned buffer laid out as the device image edgedet_jpeg_decode_batch reads (offset table, then the
    packets): uploaded with one copy, reconstructed on the device by run_batches into the plan's
    input."""

    def __init__(self, buf, span, hw, plane_bytes, n):
        self.buf, self.span, self.hw, self.plane_bytes, self.n = buf, int(span), tuple(hw), int(plane_bytes), int(n)

    def __len__(self):
        return self.n


def batch_packets(paths, threads=0, pinned=True):
    """Entropy-decode a batch of JPEG files of one size on `threads` host threads in one library call
    -> PackedBatch, or None when a file is not a JPEG the device path handles — including a non-JPEG
    file with a .jpg name and a JPEG whose entropy data the decoder rejects — or the sizes differ (the
    caller decodes the batch on the host, as read_image would).  Raises EdgeDetError only on files
    that cannot be opened or read."""
    import os
    L = ops.lib()
    n = len(paths)
    arr = (ctypes.c_char_p * n)(*[os.fsencode(p) for p in paths])
    hw = np.zeros((n, 2), np.int32)
    planes = ctypes.c_int64(0)
    # the packets run a few times the file bytes; a second call only when this guess is too small
    def size(p):
        try:
            return os.path.getsize(p)
        except OSError:  # the library reports the unreadable file
            return 0
    cap = (8 * n + 255) // 256 * 256 + sum((8 * size(p) + 65536 + 255) // 256 * 256 for p in paths)
    for _ in range(2):
        buf = torch.empty(cap, dtype=torch.uint8, pin_memory=pinned)
        span = L.edgedet_jpeg_batch_packets(ctypes.cast(arr, ctypes.c_void_p), n, buf.data_ptr(), cap,
                                            hw.ctypes.data, ctypes.byref(planes), int(threads))
        if span == 0:
            return None
        if span < 0:
            ops.check(int(span))
        if span <= cap:
            if (hw != hw[0]).any():
                return None
            return PackedBatch(buf, span, hw[0], planes.value, n)
        cap = int(span)
    raise ops.EdgeDetError("jpeg_batch_packets: packet sizes changed between two decodes of the same files")


def _nbytes(p):
    return int(p.numel()) if torch.is_tensor(p) else int(p.size)


def packet_hw(pk):
    """(H, W) of a host packet, from its header (csrc/jpeg.hip Header: magic, version, H, W, ...)."""
    head = (pk[:16].numpy() if torch.is_tensor(pk) else np.asarray(pk[:16])).view(np.int32)
    return int(head[2]), int(head[3])


def plane_bytes(pk):
    return int(ops.lib().edgedet_jpeg_plane_bytes(pk.data_ptr() if torch.is_tensor(pk) else pk.ctypes.data))


def reconstruct_host(pk, hw):
    """The host checker of the device reconstruction (csrc/jpeg.hip reconstruct_host): [3,H,W] uint8."""
    out = np.empty((3, hw[0], hw[1]), np.uint8)
    ops.check(ops.lib().edgedet_jpeg_reconstruct_host(pk.ctypes.data, out.ctypes.data))
    return out


class BatchDecoder:
    """Device reconstruction of batches of packets of one size into uint8 [B,3,H,W] device tensors.
    Keeps a pinned staging buffer and a device copy of the packets and the plane scratch, grown as
    needed; every call is asynchronous on the given stream (the caller keeps the packets' pinned
    staging alive until the stream passes the upload: decode() records an event it waits on before
    the staging is reused)."""

    def __init__(self, device):
        self.device = torch.device(device)
        self.stage = torch.empty(0, dtype=torch.uint8).pin_memory()
        self.dev = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.planes = torch.empty(0, dtype=torch.uint8, device=self.device)
        self.done = None

    def decode(self, packets, out, stream=None):
        if isinstance(packets, PackedBatch):
            return self.decode_packed(packets, out, stream)
        B, C, H, W = out.shape
        if C != 3 or out.dtype != torch.uint8 or not out.is_cuda or not out.is_contiguous() or len(packets) != B:
            raise ValueError("decode: out must be a contiguous cuda uint8 [B,3,H,W] tensor, one packet per image")
        # the colour kernel indexes every image's planes with the batch's H, W: a packet of another size
        # would make it read past that image's planes on the device
        bad = [k for k, p in enumerate(packets) if packet_hw(p) != (H, W)]
        if bad:
            raise ValueError(f"decode: packet {bad[0]} is {packet_hw(packets[bad[0]])}, the batch is {(H, W)}")
        # device image: [offsets int64, padded to 256 B][packet 0][packet 1]... (each 256-B aligned);
        # numpy packets go through one pinned staging copy, pinned tensor packets are uploaded as they are
        head = (8 * B + 255) // 256 * 256
        sizes = [_nbytes(p) for p in packets]
        direct = all(torch.is_tensor(p) and p.is_pinned() for p in packets)
        offs = np.zeros(B, np.int64)
        offs[1:] = np.cumsum([(sz + 255) // 256 * 256 for sz in sizes])[:-1]
        offs += head
        total = int(offs[-1] + sizes[-1])
        blocks = [plane_bytes(p) // 64 for p in packets]
        stride = (max(blocks) * 64 + 255) // 256 * 256
        if self.done is not None:
            self.done.synchronize()  # the previous batch's upload has left the staging buffer
        staged = head if direct else total
        if self.stage.numel() < staged:
            self.stage = torch.empty(staged * 2, dtype=torch.uint8).pin_memory()
        if self.dev.numel() < total:
            self.dev = torch.empty(total * 2, dtype=torch.uint8, device=self.device)
        if self.planes.numel() < B * stride:
            self.planes = torch.empty(B * stride * 2, dtype=torch.uint8, device=self.device)
        st = self.stage.numpy()
        st[:8 * B] = offs.view(np.uint8)
        if not direct:
            for p, o, n in zip(packets, offs, sizes):
                st[o:o + n] = p.numpy() if torch.is_tensor(p) else p
        s = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            self.dev[:staged].copy_(self.stage[:staged], non_blocking=True)
            if direct:  # the caching host allocator keeps each packet's block until its copy is done
                for p, o, n in zip(packets, offs, sizes):
                    self.dev[int(o):int(o) + n].copy_(p, non_blocking=True)
            base = self.dev.data_ptr()
            ops.check(ops.lib().edgedet_jpeg_decode_batch(ctypes.c_void_p(base), ctypes.c_void_p(base), B, H, W,
                                                           max(blocks), ctypes.c_void_p(self.planes.data_ptr()),
                                                           stride, ctypes.c_void_p(out.data_ptr()),
                                                           ops.stream_handle(s)))
            self.done = torch.cuda.Event()
            self.done.record(s)
        return out

    def decode_packed(self, pb, out, stream=None):
        """A PackedBatch: one H2D copy of its span, then the device reconstruction into out.  The
        caching host allocator keeps pb.buf's block until the copy has run."""
        B, C, H, W = out.shape
        if C != 3 or out.dtype != torch.uint8 or not out.is_cuda or not out.is_contiguous() or len(pb) != B or \
                pb.hw != (H, W):
            raise ValueError("decode: out must be a contiguous cuda uint8 [B,3,H,W] tensor of the batch's size")
        if self.dev.numel() < pb.span:
            self.dev = torch.empty(pb.span * 2, dtype=torch.uint8, device=self.device)
        stride = (pb.plane_bytes + 255) // 256 * 256
        if self.planes.numel() < B * stride:
            self.planes = torch.empty(B * stride * 2, dtype=torch.uint8, device=self.device)
        s = stream or torch.cuda.current_stream(self.device)
        with torch.cuda.stream(s):
            self.dev[:pb.span].copy_(pb.buf[:pb.span], non_blocking=True)
            base = self.dev.data_ptr()
            ops.check(ops.lib().edgedet_jpeg_decode_batch(ctypes.c_void_p(base), ctypes.c_void_p(base), B, H, W,
                                                           pb.plane_bytes // 64, ctypes.c_void_p(self.planes.data_ptr()),
                                                           stride, ctypes.c_void_p(out.data_ptr()),
                                                           ops.stream_handle(s)))
        return out
