"""MI355X-native RoCEv2 ICRC engine (drop-in for datenlord/roce-sim's
BTH.compute_icrc, src/roce.py:192-223).

Submodules:
  engine  -- ctypes binding of libroceicrc.so (HIP kernels, C ABI)
  roce    -- the reference's packet-object API (BTH, AETH, ... , IP, UDP)
             with ICRC compute/verify routed through the engine
  synth   -- synthetic frame batches for the BASELINE.json configurations
  recv    -- the receive loop: datagram sources (raw socket, pcap, memory)
             batched through the GPU ICRC verify, dispatch like recv_pkts
  hooks   -- reference-shaped SEND/RESP hooks for ICRC fault injection
"""

from .engine import (  # noqa: F401
    IcrcEngine,
    IcrcError,
    IcrcUnavailable,
    compute_batch_multi,
    verify_batch_multi,
    load_library,
    pack_aligned,
    pack_icrc,
    seg_wrs,
    segment_plan,
)
