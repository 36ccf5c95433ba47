"""Record / replay of rt_mpc_qp node traffic.

A log holds, per 100 Hz loop tick, one message row per robot:

  input log  (kind 0): /MPC/Gait (100 doubles) | /control2rtmpc/state (25)
                       = the latest message of each topic when the loop ran
                       (gait_fast.cpp:79-110 callbacks, :505 loop)
  output log (kind 1): /rtMPC/traj (100)       | /rt2nrt/state (25)
                       (gait_fast.cpp:716-734, :522-527)

File layout (little-endian): magic b"QLRTLOG1", int64 batch, int64 ticks,
int64 kind, then ticks x batch x 125 float64.  The row layout is exactly the
sensor_msgs/JointState `position` arrays of those topics, so a rosbag of the
reference's topics converts row for row (one recorded tick = the latest
message of each topic at the loop's wake-up).  Logs are memory-mapped: a
long capture never has to fit in host RAM.

    python -m quadrupedal_loco_amd.replay IN.qlog OUT.qlog [--device cuda:0]
"""
import os
import struct

import numpy as np

MAGIC = b"QLRTLOG1"
HEADER = struct.Struct("<8sqqq")
ROW = 125  # 100 + 25
KIND_INPUT, KIND_OUTPUT = 0, 1


class RtLogWriter:
    """Append-only writer; `append(a100, b25)` adds one tick (B rows)."""

    def __init__(self, path, batch, kind):
        self.path, self.batch, self.kind, self.ticks = path, int(batch), int(kind), 0
        self.f = open(path, "wb")
        self.f.write(HEADER.pack(MAGIC, self.batch, 0, self.kind))

    def append(self, a, b):
        a = np.asarray(a, np.float64).reshape(self.batch, 100)
        b = np.asarray(b, np.float64).reshape(self.batch, 25)
        self.f.write(np.ascontiguousarray(np.concatenate([a, b], axis=1)).astype("<f8").tobytes())
        self.ticks += 1

    def close(self):
        if self.f:
            self.f.seek(0)
            self.f.write(HEADER.pack(MAGIC, self.batch, self.ticks, self.kind))
            self.f.close()
            self.f = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def read_log(path):
    """-> (kind, memmap of shape (ticks, batch, 125))"""
    with open(path, "rb") as f:
        magic, batch, ticks, kind = HEADER.unpack(f.read(HEADER.size))
    if magic != MAGIC:
        raise ValueError("%s: not a qloco rt log" % path)
    size = os.path.getsize(path) - HEADER.size
    if size != ticks * batch * ROW * 8:
        raise ValueError("%s: truncated (%d bytes for %d ticks x %d robots)" % (path, size, ticks, batch))
    data = np.memmap(path, dtype="<f8", mode="r", offset=HEADER.size, shape=(ticks, batch, ROW))
    return kind, data


def replay(in_path, out_path, device="cuda:0"):
    """Drive the batched node (RtNodeBatch) with a recorded input log and write
    the output log.  Returns the number of ticks replayed."""
    import torch

    from .rt import RtNodeBatch
    kind, data = read_log(in_path)
    if kind != KIND_INPUT:
        raise ValueError("%s is not an input log" % in_path)
    ticks, batch, _ = data.shape
    dev = torch.device(device)
    node = RtNodeBatch(batch, dev)
    buf = torch.empty((batch, ROW), dtype=torch.float64, device=dev)
    with RtLogWriter(out_path, batch, KIND_OUTPUT) as w:
        for t in range(ticks):
            buf.copy_(torch.from_numpy(np.ascontiguousarray(data[t])))
            traj, nrt, _, _ = node.tick(buf[:, :100].contiguous(), buf[:, 100:].contiguous(),
                                        with_debug=False)
            w.append(traj.cpu().numpy(), nrt.cpu().numpy())
    return ticks


def main(argv=None):
    import argparse
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("input")
    ap.add_argument("output")
    ap.add_argument("--device", default="cuda:0")
    a = ap.parse_args(argv)
    n = replay(a.input, a.output, a.device)
    print("replayed %d ticks -> %s" % (n, a.output))


if __name__ == "__main__":
    main()
