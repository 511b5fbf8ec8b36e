"""Host ingest pipeline: the batched counterpart of
RecordSocket (tlslite/recordlayer.py:35-237) around the device framing of
records.py, for the bulk data of one connection direction.

* ``RecordWriter`` -- RecordLayer.sendRecord (:606-617) + _encryptThenSeal
  (:536-565) + RecordSocket.send (:83-104) for a stream of records: the
  application data is fragmented into records of at most ``send_record_limit``
  bytes (RecordLayer.send_record_limit, :316), copied into a pinned host slot,
  sealed on the GPU (tg_seal_records: header, TLS 1.2 explicit nonce, TLS 1.3
  inner type + padding, AEAD), packed into one contiguous wire stream on the
  device (tg_gather) and copied back to a pinned buffer that goes to the sink's
  ``sendall``.
* ``RecordReader`` -- RecordSocket.recv (:207-237) + RecordLayer.recvRecord /
  _decryptAndUnseal (:780-824) / _tls13_de_pad (:863-884): wire bytes are
  accumulated in a pinned buffer, the complete records are found by
  tg_scan_records (host C, with RecordSocket's length limits), copied to the
  device in one piece, spread into 16-byte aligned slots (tg_gather), opened
  (tg_open_records) and returned in order as ``(content_type, bytearray)``;
  the first failing record raises the reference's exception.

Each direction keeps ``nslots`` slots (3 by default), each with its own HIP
stream: while one batch runs host->device copy, kernels and device->host
copy, the host fills the next slot (writer); the reader's bulk path opens
batch k+1 while batch k is packed and copied back (both PCIe directions busy
at once).  Sequence numbers run on from ``seq0`` as in
ConnectionState.getSeqNumBytes (:251-256).

Host copies (application data into the writer's pinned slot, socket bytes
into the reader's pinned buffer) go through ``tg_host_copy``: split over a
pool of native threads, the GIL released.  Callers that can produce the
bytes in place skip the copy: ``RecordWriter.write_buffer`` / ``commit``
hand out the pinned slot itself, ``RecordReader.recv_buffer`` / ``commit``
the reader's pinned buffer (e.g. for ``socket.recv_into``).  And
``RecordReader.read_application_data(out, data=...)`` copies the socket bytes
batch by batch while the batches before run on the GPU.
"""
import ctypes

import numpy as np

from . import _lib
from .batch import _ptr
from .records import TLS12, TLS13, open_records, seal_records


class TLSProtocolException(Exception):
    """tlslite.errors.TLSProtocolException (errors.py:195)."""


class TLSIllegalParameterException(TLSProtocolException):
    """errors.py:201"""


class TLSUnexpectedMessage(TLSProtocolException):
    """errors.py:213"""


class TLSRecordOverflow(TLSProtocolException):
    """errors.py:222"""


class TLSBadRecordMAC(TLSProtocolException):
    """errors.py:234"""


# tg_open_records status -> the exception _decryptAndUnseal / _tls13_de_pad raise
_STATUS_EXC = {
    1: (TLSBadRecordMAC, "Invalid tag, decryption failure"),
    2: (TLSBadRecordMAC, "Truncated tag"),
    3: (TLSBadRecordMAC, "Length mismatch"),
    4: (TLSUnexpectedMessage, "Invalid ContentType for encrypted record"),
    5: (TLSIllegalParameterException, "Unexpected version in encrypted record"),
    6: (TLSUnexpectedMessage, "Malformed record layer inner plaintext - content type missing"),
    7: (TLSRecordOverflow, "Record over the receive limit"),
}

APPLICATION_DATA = 23


def _ru(x, m):
    return (x + m - 1) // m * m


# threads of the host copies (tg_host_copy; 0 = the library's default); the
# GPU box gives a process 16 cores
COPY_THREADS = 12


def _addr(a):
    """Host address of a numpy array / pinned CPU tensor."""
    return a.ctypes.data if isinstance(a, np.ndarray) else a.data_ptr()


def host_copy(dst, src, nbytes=None):
    """dst[:n] = src[:n] for host numpy arrays (or pinned CPU tensors) through
    tg_host_copy: native threads, GIL released."""
    n = len(src) if nbytes is None else int(nbytes)
    if n == 0:
        return
    _lib.check(_lib.load().tg_host_copy(_addr(dst), _addr(src), n, COPY_THREADS))


def _explicit_nonce(version, key):
    # TLS 1.2 AES-GCM / AES-CCM carry an 8-byte explicit nonce ("aes" in name)
    return 8 if version == TLS12 and "aes" in key.name else 0


class _Slot(object):
    """Pinned host + device buffers and a stream for one batch in flight."""

    def __init__(self, torch, nrec, data_stride, wire_stride, wire_lead, app_bytes=0):
        self.stream = torch.cuda.Stream()
        self.event = torch.cuda.Event()
        self.app_event = torch.cuda.Event()   # the writer's h_app has gone to the device
        self.busy = False        # wire output of the slot's last launch not yet sent
        self.filling = False     # the writer's h_app still in use by a launch
        u8 = torch.uint8
        self.h_data = torch.empty(nrec * data_stride, dtype=u8).pin_memory()
        self.h_wire = torch.empty(nrec * wire_stride, dtype=u8).pin_memory()
        self.d_data = torch.empty(nrec * data_stride, dtype=u8, device="cuda")
        self.d_wire = torch.empty(nrec * wire_stride + 16, dtype=u8, device="cuda")
        self.d_pack = torch.empty(nrec * wire_stride, dtype=u8, device="cuda")
        # per-record metadata: one pinned host block and one device block with
        # the same layout, so each direction moves it in ONE copy per batch
        # (small copies run as blit kernels at ~5 us each, plus the host's
        # launch overhead):
        #   P int64 @0     pack offsets          S int64 @8n   writer app / reader wire offsets
        #   L int32 @16n   lengths               R int32 @20n  reader wire lengths / writer wire lengths
        #   Q int32 @24n   reader packed lengths T u8 @28n     content types     U u8 @29n  status
        self.nrec = nrec
        self.h_meta = torch.empty(32 * nrec, dtype=u8).pin_memory()
        self.d_meta = torch.empty(32 * nrec, dtype=u8, device="cuda")

        def views(m):
            n = nrec
            return (m[0:8 * n].view(torch.int64), m[8 * n:16 * n].view(torch.int64),
                    m[16 * n:20 * n].view(torch.int32), m[20 * n:24 * n].view(torch.int32),
                    m[24 * n:28 * n].view(torch.int32), m[28 * n:29 * n], m[29 * n:30 * n])
        (self.h_pack, self.h_src, self.h_len, self.h_rl, self.h_plen, self.h_ctype,
         self.h_status) = views(self.h_meta)
        (self.d_pack_off, self.d_src, self.d_len, self.d_wlen, self.d_plen, self.d_ctype,
         self.d_status) = views(self.d_meta)
        self.d_rl = self.d_wlen
        self.h_app_off, self.d_app_off = self.h_src, self.d_src
        idx = torch.arange(nrec, dtype=torch.int64, device="cuda")
        self.d_data_off = idx * data_stride
        self.d_wire_off = idx * wire_stride + wire_lead
        if app_bytes:   # the writer's application data, contiguous
            self.h_app = torch.empty(app_bytes, dtype=u8).pin_memory()
            self.d_app = torch.empty(app_bytes, dtype=u8, device="cuda")
        self.n = 0
        self.nbytes = 0
        self.app = 0

    # metadata rows in units of nrec bytes: P [0, 8), S [8, 16), L [16, 20),
    # R [20, 24), Q [24, 28), T [28, 29), U [29, 30)
    def meta_to_device(self, lo, hi):
        n = self.nrec
        self.d_meta[lo * n:hi * n].copy_(self.h_meta[lo * n:hi * n], non_blocking=True)

    def meta_to_host(self, lo, hi):
        n = self.nrec
        self.h_meta[lo * n:hi * n].copy_(self.d_meta[lo * n:hi * n], non_blocking=True)


class RecordWriter(object):
    """Seal and send a stream of records of one connection direction.

    :param sink: object with ``sendall(buffer)`` (a socket, or any byte sink)
    :param key: the direction's AEAD object (HipAESGCM / HipAESCCM /
        HipCHACHA20_POLY1305, i.e. ConnectionState.encContext)
    :param version: TLS12 or TLS13 (records.py)
    :param fixed_iv: ConnectionState.fixedNonce (12 bytes, or 4 for TLS 1.2
        AES-GCM / AES-CCM)

    A slot holds the application data of up to ``batch_records`` records
    contiguously in pinned memory; at launch it goes to the device in one
    copy, is spread into the 16-byte aligned rows that tg_seal_records seals
    in place (tg_gather), sealed, packed into one wire stream and copied
    back.
    """

    def __init__(self, sink, key, version, fixed_iv, seq0=0, send_record_limit=2 ** 14,
                 batch_records=1024, nslots=3, pad=0):
        import torch
        if version not in (TLS12, TLS13):
            raise ValueError("version must be TLS12 or TLS13")
        self.torch = torch
        self.sink = sink
        self.key = key
        self.version = version
        self.fixed_iv = bytes(fixed_iv)
        self.seq = int(seq0)
        self.limit = int(send_record_limit)
        self.pad = int(pad) if version == TLS13 else 0
        self.batch = int(batch_records)
        self.hdr = 5 + _explicit_nonce(version, key)
        self.tag = key.tagLength
        inner = self.limit + (1 + self.pad if version == TLS13 else 0)
        self.data_stride = _ru(inner + 16, 16)
        # payload after header (+ explicit nonce) starts 16-byte aligned
        self.lead = _ru(self.hdr, 16) - self.hdr
        self.wire_stride = _ru(self.lead + self.hdr + inner + self.tag, 16)
        self.app_cap = self.batch * self.limit
        self.slots = [_Slot(torch, self.batch, self.data_stride, self.wire_stride, self.lead,
                            app_bytes=self.app_cap) for _ in range(nslots)]
        self.cur = 0
        self.records_sent = 0
        self.bytes_sent = 0

    def _slot(self):
        """The slot being filled.  Its h_app may be refilled once the copy of
        its last launch's application data to the device has finished; its
        wire output of that launch is sent before its next launch."""
        s = self.slots[self.cur]
        if s.filling:
            s.app_event.synchronize()
            s.filling = False
        return s

    def _records(self, s, nbytes, content_type):
        """Cut nbytes of application data, just placed at s.h_app[s.app:],
        into records of at most send_record_limit bytes (sendRecord per
        write call)."""
        k = min(-(-nbytes // self.limit), self.batch - s.n) if nbytes else 1
        lens = np.full(k, self.limit, np.int32)
        if nbytes:
            lens[-1] = nbytes - (k - 1) * self.limit
        else:
            lens[0] = 0
        offs = s.app + np.arange(k, dtype=np.int64) * self.limit
        s.h_len.numpy()[s.n:s.n + k] = lens
        s.h_ctype.numpy()[s.n:s.n + k] = content_type
        s.h_app_off.numpy()[s.n:s.n + k] = offs
        s.n += k
        s.app += nbytes
        if s.n == self.batch or s.app + self.limit > self.app_cap:
            self._launch(s)

    # -- RecordLayer.sendRecord for application data, batched
    def write(self, data, content_type=APPLICATION_DATA):
        """Queue ``data`` as records of at most send_record_limit bytes (an
        empty ``data`` queues one empty record, as sendRecord does)."""
        mv = memoryview(bytes(data) if not isinstance(data, (bytes, bytearray, memoryview))
                        else data).cast("B")
        src = np.frombuffer(mv, np.uint8)
        pos = 0
        while True:
            s = self._slot()
            # whole records while the slot has room: one (threaded) copy
            room = min((self.batch - s.n) * self.limit, self.app_cap - s.app)
            k = min(len(src) - pos, room)
            if k:
                host_copy(s.h_app.numpy()[s.app:], src[pos:], k)
            self._records(s, k, content_type)
            pos += k
            if pos >= len(src):
                break

    def write_buffer(self):
        """Zero-copy write: a writable memoryview of the current slot's free
        pinned space (at least one record's worth).  Put application data at
        its start, then call ``commit(n)``."""
        s = self._slot()
        room = min((self.batch - s.n) * self.limit, self.app_cap - s.app)
        return memoryview(s.h_app.numpy()[s.app:s.app + room])

    def commit(self, nbytes, content_type=APPLICATION_DATA):
        """Queue the ``nbytes`` bytes placed at the start of write_buffer()
        as records (as write() would)."""
        s = self.slots[self.cur]
        room = min((self.batch - s.n) * self.limit, self.app_cap - s.app)
        if s.filling or not 0 <= nbytes <= room:
            raise ValueError("commit() without a matching write_buffer(), or too many bytes")
        self._records(s, int(nbytes), content_type)

    def flush(self):
        """Seal what is queued and send everything in order."""
        s = self._slot()
        if s.n:
            self._launch(s)
        # the slot after the last launched one holds the oldest unsent output
        for k in range(len(self.slots)):
            s = self.slots[(self.cur + k) % len(self.slots)]
            if s.busy:
                self._finish(s)

    def _wire_len(self, L):
        inner = L + (1 + self.pad if self.version == TLS13 else 0)
        return self.hdr + inner + self.tag

    def _launch(self, s):
        torch = self.torch
        if s.busy:   # its previous wire output goes out first (in launch order)
            self._finish(s)
        n = s.n
        lens = s.h_len.numpy()[:n].astype(np.int64)
        wl = self._wire_len(lens)
        pack = s.h_pack.numpy()
        pack[0] = 0
        if n > 1:
            np.cumsum(wl[:-1], out=pack[1:n])
        s.nbytes = int(wl.sum())
        pad = None
        with torch.cuda.stream(s.stream):
            if s.app:
                s.d_app[:s.app].copy_(s.h_app[:s.app], non_blocking=True)
            s.meta_to_device(0, 29)        # pack and app offsets, lengths, types (R: seal's output)
            s.app_event.record(s.stream)   # h_app and the row metadata may be refilled
            # the fragments into their aligned rows (room for the inner type,
            # padding and tag after each)
            gather(s.d_app, s.d_app_off, s.d_len, s.d_data, s.d_data_off, n, stream=s.stream)
            if self.pad:
                pad = torch.full((n,), self.pad, dtype=torch.int32, device="cuda")
            seal_records(self.key, self.version, self.fixed_iv, self.seq, n, s.d_data, s.d_data_off,
                         s.d_len, s.d_ctype, s.d_wire, s.d_wire_off, s.d_wlen, pad_len=pad,
                         stream=s.stream)
            gather(s.d_wire, s.d_wire_off, s.d_wlen, s.d_pack, s.d_pack_off, n, stream=s.stream)
            s.h_wire[:s.nbytes].copy_(s.d_pack[:s.nbytes], non_blocking=True)
            s.event.record(s.stream)
        s.keep = pad
        s.busy = True
        s.filling = True
        s.sent_n, s.n, s.app = n, 0, 0
        self.seq += n
        self.cur = (self.cur + 1) % len(self.slots)

    def _finish(self, s):
        s.event.synchronize()
        self.sink.sendall(memoryview(s.h_wire.numpy())[:s.nbytes])
        self.records_sent += s.sent_n
        self.bytes_sent += s.nbytes
        s.busy = False


class RecordReader(object):
    """Receive, check and open a stream of records of one connection
    direction (wire bytes in, ``(content_type, bytearray)`` out).

    ``feed(wire_bytes)`` queues bytes as they come off the socket;
    ``records()`` returns the records completed so far, in order.  Errors:
    TLSRecordOverflow / TLSIllegalParameterException for a bad header
    (RecordSocket.recv), then per record the exception _decryptAndUnseal or
    _tls13_de_pad would raise; records before the failing one are returned
    by ``records()`` first and the error is raised on the next call.
    """

    def __init__(self, key, version, fixed_iv, seq0=0, recv_record_limit=2 ** 14,
                 batch_records=1024, buffer_bytes=None, nslots=3):
        import torch
        if version not in (TLS12, TLS13):
            raise ValueError("version must be TLS12 or TLS13")
        self.torch = torch
        self.key = key
        self.version = version
        self.fixed_iv = bytes(fixed_iv)
        self.seq = int(seq0)
        # RecordSocket.recv (:217-222): 2**14 + 2048 always, 2**14 + 256 for TLS 1.3
        self.recv_record_limit = int(recv_record_limit)
        self.max_body = recv_record_limit + (256 if version == TLS13 else 2048)
        self.batch = int(batch_records)
        self.hdr = 5 + _explicit_nonce(version, key)
        self.lead = _ru(self.hdr, 16) - self.hdr
        self.wire_stride = _ru(self.lead + 5 + self.max_body, 16)
        self.data_stride = _ru(self.max_body + 16, 16)
        cap = buffer_bytes or self.batch * (5 + self.max_body)
        self.h_buf = torch.empty(cap, dtype=torch.uint8).pin_memory()
        self.fill = 0
        self.slot = _Slot(torch, self.batch, self.data_stride, self.wire_stride, self.lead)
        self.h_off = np.empty(self.batch, np.uint64)
        self.h_rlen = np.empty(self.batch, np.uint32)
        self.h_out = torch.empty(self.batch * self.data_stride, dtype=torch.uint8).pin_memory()
        # the pipelined bulk path (read_application_data): per-slot gather indices
        self.rslots = [self.slot] + [_Slot(torch, self.batch, self.data_stride, self.wire_stride,
                                           self.lead) for _ in range(max(1, nslots) - 1)]
        self.pending_error = None
        self._pool = None

    def _reserve(self, nbytes):
        """Room for nbytes more in the pinned buffer (grows it if needed)."""
        need = self.fill + nbytes
        if need > self.h_buf.numel():
            nb = self.torch.empty(max(need, 2 * self.h_buf.numel()), dtype=self.torch.uint8).pin_memory()
            host_copy(nb.numpy(), self.h_buf.numpy(), self.fill)
            self.h_buf = nb

    def feed(self, data):
        """Append wire bytes (grows the pinned buffer if needed)."""
        mv = memoryview(data).cast("B")
        self._reserve(len(mv))
        host_copy(self.h_buf.numpy()[self.fill:], np.frombuffer(mv, np.uint8), len(mv))
        self.fill += len(mv)

    def recv_buffer(self, nbytes=1 << 20):
        """Zero-copy feed: a writable memoryview of at least ``nbytes`` free
        bytes of the pinned buffer, e.g. for ``sock.recv_into``; then
        ``commit(n)`` with the bytes received."""
        self._reserve(nbytes)
        return memoryview(self.h_buf.numpy()[self.fill:])

    def commit(self, nbytes):
        """Account ``nbytes`` bytes written at the start of recv_buffer()."""
        if not 0 <= nbytes <= self.h_buf.numel() - self.fill:
            raise ValueError("commit() beyond the buffer")
        self.fill += int(nbytes)

    def _scan(self, start=0):
        """tg_scan_records over h_buf[start:fill]: (records, bytes, error)."""
        lib = _lib.load()
        consumed = ctypes.c_size_t(0)
        buf = self.h_buf.numpy()[start:]
        rc = lib.tg_scan_records(buf.ctypes.data, self.fill - start, self.max_body,
                                 self.h_off.ctypes.data, self.h_rlen.ctypes.data, self.batch,
                                 ctypes.byref(consumed))
        if rc == _lib.TG_EOVERFLOW:
            n = _count(self.h_rlen, consumed.value)
            return n, consumed.value, TLSRecordOverflow()
        if rc == _lib.TG_EHEADER:
            n = _count(self.h_rlen, consumed.value)
            return n, consumed.value, TLSIllegalParameterException("Malformed record layer header")
        _lib.check(rc)
        return int(rc), consumed.value, None

    def records(self):
        """Open every complete record fed so far; returns [(type, bytearray)]."""
        out = []
        for ct, plen in self._batches():
            if len(plen) == 0:
                continue
            ho = self._rows_to_host(len(plen))
            for i in range(len(plen)):
                o = i * self.data_stride
                out.append((int(ct[i]), bytearray(ho[o:o + int(plen[i])].tobytes())))
        return out

    def read_application_data(self, out=None, data=None):
        """The bulk path: the plaintext of every application-data record
        completed so far, concatenated (other content types are dropped, as a
        caller that reads only application data would), copied into ``out``
        (a writable buffer, filled from offset 0) or a new bytearray; returns
        that buffer's filled part (memoryview / bytearray).  Raises like
        records().

        ``data``: wire bytes to feed first (as feed(data)), copied into the
        pinned buffer a batch at a time while the batches before it are
        opened and copied back, so the host copy overlaps the GPU work.

        Pipelined over ``nslots`` slots, each with its own stream: batch k+1's
        H2D copy and open run while batch k is packed on the device
        (tg_gather of its application-data plaintexts) and copied back, so the
        PCIe directions overlap.  When ``out`` is pinned host memory (e.g. the
        numpy view of a pinned torch tensor) the packed bytes land in it
        directly and the host never waits for them; otherwise HIP stages the
        copy (the host waits for it while the next batch is already queued)."""
        if self.pending_error is not None:
            e, self.pending_error = self.pending_error, None
            raise e
        torch = self.torch
        dst = None if out is None else np.frombuffer(out, np.uint8)
        direct = dst is not None and len(dst) > 0 and torch.from_numpy(dst[:1]).is_pinned()
        src, spos = None, 0
        if data is not None:
            src = np.frombuffer(memoryview(data).cast("B"), np.uint8)
            self._reserve(len(src))      # no reallocation while copies from h_buf run
        # bytes of wire data per batch the scan should have in front of it
        chunk = self.batch * (5 + self.max_body)
        fill_entry = self.fill
        pieces = []
        self._pos = 0
        self._got = False
        self._dead = False
        seq_entry = self.seq
        meta, done = [], []        # slots opened (metadata pending) / packed (copy pending)
        free = list(self.rslots)
        start = 0
        err = None
        # ``data`` goes into the pinned buffer one chunk ahead, on a helper
        # thread (tg_host_copy releases the GIL), while this thread scans,
        # launches and waits for the batches before it
        pend = None       # (future, bytes) of the chunk being copied to h_buf[fill:]

        def kick():
            nonlocal spos, pend
            if pend is None and src is not None and spos < len(src):
                k = min(len(src) - spos, chunk)
                pend = (self._copier().submit(host_copy, self.h_buf.numpy()[self.fill:], src[spos:], k), k)
                spos += k

        try:
            while not self._dead:
                kick()
                if pend is not None and self.fill - start < chunk:
                    pend[0].result()
                    self.fill += pend[1]
                    pend = None
                    continue
                n, used, err = self._scan(start)
                if n:
                    if not free:
                        if not done:
                            done.append(self._pack(meta.pop(0), dst, direct, pieces))
                        free.append(self._finish_read(done.pop(0), dst))
                    s = free.pop(0)
                    self._enqueue_open(s, start, n, used)
                    start += used
                    meta.append(s)
                    if len(meta) > 1:
                        done.append(self._pack(meta.pop(0), dst, direct, pieces))
                if err is not None or (n < self.batch and pend is None and (src is None or spos >= len(src))):
                    break
            while meta:
                done.append(self._pack(meta.pop(0), dst, direct, pieces))
        except _OutTooSmall:
            if pend is not None:
                pend[0].result()
            # nothing of this call is delivered: wait for every slot still
            # running (opens, and copies into ``out``), then undo the call --
            # the sequence number and the wire bytes stay where they were, so
            # a retry with a larger buffer returns the same bytes
            for s in meta + done + self.rslots:
                s.event.synchronize()
            self.seq = seq_entry
            self.fill = fill_entry     # ``data`` was not consumed either
            self.pending_error = None
            self._dead = False
            raise ValueError("output buffer too small")
        if pend is not None:   # (an error ended the loop with a chunk in flight)
            pend[0].result()
            self.fill += pend[1]
        while done:
            self._finish_read(done.pop(0), dst)
        # the unconsumed tail to the front (every copy from h_buf has finished)
        if self._dead:
            self.fill = 0
        else:
            tail = self.fill - start
            if tail and start:
                buf = self.h_buf.numpy()
                buf[:tail] = buf[start:self.fill].copy()
            self.fill = tail
        if err is not None and not self._dead:
            self.fill = 0
            self.pending_error = err
        # an error with no record before it is raised now, else on the next call
        if self.pending_error is not None and not self._got:
            e, self.pending_error = self.pending_error, None
            raise e
        if dst is not None:
            return memoryview(out)[:self._pos]
        if len(pieces) == 1:
            return pieces[0]
        return bytearray(b"".join(pieces))

    def _copier(self):
        if self._pool is None:
            import concurrent.futures
            self._pool = concurrent.futures.ThreadPoolExecutor(1, thread_name_prefix="tlsgpu-recv")
        return self._pool

    def _enqueue_open(self, s, start, n, used):
        """H2D of n scanned records (wire bytes h_buf[start:start+used]),
        spread into aligned slots, tg_open_records, metadata back; async on
        the slot's stream.  The slot's sequence number is s.seq."""
        torch = self.torch
        src = s.h_src.numpy()
        src[:n] = self.h_off[:n].astype(np.int64)
        s.h_rl.numpy()[:n] = self.h_rlen[:n].astype(np.int32)
        s.n = n
        s.seq = self.seq
        self.seq += n
        with torch.cuda.stream(s.stream):
            s.d_pack[:used].copy_(self.h_buf[start:start + used], non_blocking=True)
            s.meta_to_device(8, 24)        # wire offsets and lengths (L: open's output)
            gather(s.d_pack, s.d_src, s.d_rl, s.d_wire, s.d_wire_off, n, stream=s.stream)
            open_records(self.key, self.version, self.fixed_iv, s.seq, n, s.d_wire,
                         s.d_wire_off, s.d_rl, s.d_data, s.d_data_off, s.d_len, s.d_ctype,
                         s.d_status, stream=s.stream, recv_limit=self.recv_record_limit)
            s.meta_to_host(16, 30)         # lengths, types, status (R and Q come back unchanged)
            s.event.record(s.stream)

    def _pack(self, s, dst, direct, pieces):
        """Wait for slot s's metadata; pack its application-data plaintexts
        (records before the first failing one) on the device and start the
        copy back to ``dst`` (or a new piece when ``dst`` is None)."""
        torch = self.torch
        s.event.synchronize()
        s.total = 0
        s.target = None
        if self._dead:
            return s
        n = s.n
        st = s.h_status.numpy()[:n]
        bad = np.nonzero(st)[0]
        k = int(bad[0]) if len(bad) else n
        if len(bad):
            cls, msg = _STATUS_EXC.get(int(st[k]), (TLSProtocolException, "record error"))
            self.pending_error = cls(msg)
            self._dead = True
            self.seq = s.seq + k           # later slots were opened past the failure
        self._got = self._got or k > 0
        ct = s.h_ctype.numpy()[:k]
        L = s.h_len.numpy()[:k].astype(np.int64) * (ct == APPLICATION_DATA)
        total = int(L.sum())
        s.total = total
        if total == 0:
            return s
        off = s.h_pack.numpy()
        off[0] = 0
        if k > 1:
            np.cumsum(L[:-1], out=off[1:k])
        s.h_plen.numpy()[:k] = L.astype(np.int32)
        if dst is not None:
            if self._pos + total > len(dst):
                raise _OutTooSmall()
            s.target = (self._pos, total)
        else:
            piece = bytearray(total)
            pieces.append(piece)
            s.target = piece
        with torch.cuda.stream(s.stream):
            s.meta_to_device(0, 28)        # pack offsets and packed lengths (S, L, R as uploaded / read)
            gather(s.d_data, s.d_data_off, s.d_plen, s.d_pack, s.d_pack_off, k, stream=s.stream)
            if isinstance(s.target, bytearray):
                tgt = np.frombuffer(s.target, np.uint8)
            else:
                tgt = dst[self._pos:self._pos + total]
            # pinned: an async DMA; pageable: HIP's staged copy (blocks the host,
            # the next batch's open is already queued on its own stream)
            torch.from_numpy(tgt).copy_(s.d_pack[:total], non_blocking=direct)
            s.event.record(s.stream)
        self._pos += total
        return s

    def _finish_read(self, s, dst):
        """Wait for slot s's copy back."""
        s.event.synchronize()
        s.n = 0
        return s

    def _batches(self):
        """Open the complete records batch by batch; yields (ctype, plen) per
        batch, the plaintexts in the slot's device rows.  An error stops at the failing record: the
        records before it are yielded, the exception is raised on the next
        call (at once if there were none)."""
        if self.pending_error is not None:
            e, self.pending_error = self.pending_error, None
            raise e
        got = False
        while True:
            n, used, err = self._scan()
            if n:
                res = self._open(n, used)
                got = got or len(res[1]) > 0
                yield res
                if self.pending_error is not None:
                    if not got:
                        e, self.pending_error = self.pending_error, None
                        raise e
                    return
            if err is not None:
                self.fill = 0
                if got:
                    self.pending_error = err
                    return
                raise err
            if n < self.batch:
                return

    def _open(self, n, used):
        """Open n scanned records on the device; the plaintexts stay in the
        slot's device rows (i * data_stride).  Returns (ctype, plen) of the
        records before the first failing one (whose error is kept pending)."""
        torch = self.torch
        s = self.slot
        s.h_src.numpy()[:n] = self.h_off[:n].astype(np.int64)
        s.h_rl.numpy()[:n] = self.h_rlen[:n].astype(np.int32)
        with torch.cuda.stream(s.stream):
            s.d_pack[:used].copy_(self.h_buf[:used], non_blocking=True)
            s.meta_to_device(8, 24)
            # wire records into 16-byte aligned slots (payload after header aligned)
            gather(s.d_pack, s.d_src, s.d_rl, s.d_wire, s.d_wire_off, n, stream=s.stream)
            open_records(self.key, self.version, self.fixed_iv, self.seq, n, s.d_wire,
                         s.d_wire_off, s.d_rl, s.d_data, s.d_data_off, s.d_len, s.d_ctype,
                         s.d_status, stream=s.stream, recv_limit=self.recv_record_limit)
            s.meta_to_host(16, 30)
            s.event.record(s.stream)
        s.event.synchronize()
        # the unconsumed tail to the front (the copy above has read h_buf)
        tail = self.fill - used
        if tail:
            buf = self.h_buf.numpy()
            buf[:tail] = buf[used:self.fill].copy()
        self.fill = tail
        st = s.h_status.numpy()[:n]
        plen = s.h_len.numpy()[:n]
        ct = s.h_ctype.numpy()[:n]
        bad = np.nonzero(st)[0]
        k = int(bad[0]) if len(bad) else n
        if len(bad):
            cls, msg = _STATUS_EXC.get(int(st[k]), (TLSProtocolException, "record error"))
            self.pending_error = cls(msg)
            self.fill = 0
        self.seq += k
        return ct[:k].copy(), plen[:k].copy()

    def _rows_to_host(self, k):
        """Device plaintext rows 0..k-1 -> h_out (pinned), same layout."""
        s = self.slot
        span = (k - 1) * self.data_stride + self.max_body
        with self.torch.cuda.stream(s.stream):
            self.h_out[:span].copy_(s.d_data[:span], non_blocking=True)
        s.stream.synchronize()
        return self.h_out.numpy()


class _OutTooSmall(Exception):
    """read_application_data: the caller's buffer cannot take a batch."""


def read_application_data(reader):
    """RecordReader.read_application_data (module-level alias)."""
    return reader.read_application_data()


def _count(rlen, consumed):
    n, tot = 0, 0
    while tot < consumed:
        tot += int(rlen[n])
        n += 1
    return n


def gather(src, src_off, lens, dst, dst_off, n, stream=None):
    """tg_gather: copy n byte ranges src[src_off[i]:+len[i]] -> dst[dst_off[i]:]."""
    from .batch import _stream
    l = _lib.load()
    _lib.check(l.tg_gather(_ptr(src, "src"), _ptr(src_off, "src_off"), _ptr(lens, "len"),
                           _ptr(dst, "dst"), _ptr(dst_off, "dst_off"), int(n), _stream(stream)))


def scan_records(buf, max_body, max_n=None):
    """tg_scan_records on a host buffer: ([(offset, record_len)], consumed);
    raises TLSRecordOverflow / TLSIllegalParameterException like RecordSocket."""
    a = np.frombuffer(bytes(buf), np.uint8)
    max_n = max_n if max_n is not None else max(1, len(a) // 5)
    off = np.empty(max_n, np.uint64)
    rl = np.empty(max_n, np.uint32)
    consumed = ctypes.c_size_t(0)
    rc = _lib.load().tg_scan_records(a.ctypes.data if len(a) else None, len(a), int(max_body),
                                     off.ctypes.data, rl.ctypes.data, max_n, ctypes.byref(consumed))
    if rc == _lib.TG_EOVERFLOW:
        raise TLSRecordOverflow()
    if rc == _lib.TG_EHEADER:
        raise TLSIllegalParameterException("Malformed record layer header")
    _lib.check(rc)
    return [(int(off[i]), int(rl[i])) for i in range(rc)], consumed.value
