"""Generate tests/golden/{frames.bin, vectors.json}: ICRC golden vectors.

Run in the development container: ``python tests/golden/gen_golden.py``.

What the vectors are ("Golden vectors to generate"):
  1. every RC opcode shape the simulator emits (src/roce_sq.py:1243-1466,
     src/roce_rq.py:388-525 and 767-854) with payloads that exercise padcount
     0..3 and PMTU 256 .. 4096;
  2. the ``sim_send_success`` SEND_ONLY of BASELINE config 1;
  3. mask-invariance pairs: masked fields randomised, same ICRC;
  4. non-mask sensitivity: one bit flipped in IP id/flags, pkey, resv7,
     ackreq or payload, different ICRC;
  5. IPv4-with-options and non-IPv4/UDP frames (reference warning path, ICRC 0).

Expected values come from the oracle's zlib.crc32 restatement of
BTH.compute_icrc (src/roce.py:192-223) and are cross-checked here against the
independent bitwise CRC seeded 0xDEBB20E3.  They are NOT reference-executed
(scapy is absent, see oracle/icrc_oracle.py), i.e. regression fixtures that pin
the restatement, with the CRC arithmetic itself pinned to zlib.
"""
import json
import random
import sys
from pathlib import Path

HERE = Path(__file__).resolve().parent
sys.path.insert(0, str(HERE.parent.parent / "oracle"))
import icrc_oracle as o  # noqa: E402

RC_SHAPES = {
    # opcode: (name, ext header builder, carries payload)
    0x00: ("SEND_FIRST", lambda r: b"", True),
    0x01: ("SEND_MIDDLE", lambda r: b"", True),
    0x02: ("SEND_LAST", lambda r: b"", True),
    0x03: ("SEND_LAST_WITH_IMMEDIATE", lambda r: o.immdt_bytes(r.getrandbits(32)), True),
    0x04: ("SEND_ONLY", lambda r: b"", True),
    0x05: ("SEND_ONLY_WITH_IMMEDIATE", lambda r: o.immdt_bytes(r.getrandbits(32)), True),
    0x06: ("RDMA_WRITE_FIRST", lambda r: o.reth_bytes(r.getrandbits(64), r.getrandbits(32), 8192), True),
    0x07: ("RDMA_WRITE_MIDDLE", lambda r: b"", True),
    0x08: ("RDMA_WRITE_LAST", lambda r: b"", True),
    0x09: ("RDMA_WRITE_LAST_WITH_IMMEDIATE", lambda r: o.immdt_bytes(r.getrandbits(32)), True),
    0x0A: ("RDMA_WRITE_ONLY", lambda r: o.reth_bytes(r.getrandbits(64), r.getrandbits(32), 100), True),
    0x0B: ("RDMA_WRITE_ONLY_WITH_IMMEDIATE",
           lambda r: o.reth_immdt_bytes(r.getrandbits(64), r.getrandbits(32), 10, r.getrandbits(32)), True),
    0x0C: ("RDMA_READ_REQUEST", lambda r: o.reth_bytes(r.getrandbits(64), r.getrandbits(32), 4096), False),
    0x0D: ("RDMA_READ_RESPONSE_FIRST", lambda r: o.aeth_bytes(0, 31, r.getrandbits(24)), True),
    0x0E: ("RDMA_READ_RESPONSE_MIDDLE", lambda r: b"", True),
    0x0F: ("RDMA_READ_RESPONSE_LAST", lambda r: o.aeth_bytes(0, 31, r.getrandbits(24)), True),
    0x10: ("RDMA_READ_RESPONSE_ONLY", lambda r: o.aeth_bytes(0, 31, r.getrandbits(24)), True),
    0x11: ("ACKNOWLEDGE", lambda r: o.aeth_bytes(r.choice([0, 1, 3]), r.getrandbits(5), r.getrandbits(24)), False),
    0x12: ("ATOMIC_ACKNOWLEDGE",
           lambda r: o.aeth_bytes(0, 31, r.getrandbits(24)) + o.atomic_ack_eth_bytes(r.getrandbits(64)), False),
    0x13: ("COMPARE_SWAP",
           lambda r: o.atomic_eth_bytes(r.getrandbits(64), r.getrandbits(32), r.getrandbits(64), r.getrandbits(64)), False),
    0x14: ("FETCH_ADD",
           lambda r: o.atomic_eth_bytes(r.getrandbits(64), r.getrandbits(32), 0, r.getrandbits(64)), False),
    0x16: ("SEND_LAST_WITH_INVALIDATE", lambda r: o.ieth_bytes(r.getrandbits(32)), True),
    0x17: ("SEND_ONLY_WITH_INVALIDATE", lambda r: o.ieth_bytes(r.getrandbits(32)), True),
    0x81: ("CNP", lambda r: o.cnp_padding_bytes(), False),
}
PAYLOAD_LENS = [0, 1, 2, 3, 4, 5, 6, 7, 255, 256, 512, 1024, 2048, 4096]


def main():
    rnd = random.Random(0x1C2C0000)
    vectors, blob = [], bytearray()

    def add(name, frame, **meta):
        expect = o.icrc_of_frame(frame)
        assert expect == o.icrc_bitwise(frame), name  # independent cross-check
        vectors.append(dict(name=name, offset=len(blob), len=len(frame),
                            icrc=f"{expect:08x}", **meta))
        blob.extend(frame)
        blob.extend(b"\0" * ((-len(frame)) % 4))

    f = o.sim_send_success_frame()
    add("cfg1_sim_send_success", f, kind="config1")
    for op, (nm, ext, has_pay) in RC_SHAPES.items():
        for pl in (PAYLOAD_LENS if has_pay else [None]):
            if pl is not None and pl > 256 and op not in (0x01, 0x04, 0x07, 0x0E):
                continue
            payload = None if pl is None else bytes(rnd.getrandbits(8) for _ in range(pl))
            bth = dict(opcode=op, psn=rnd.getrandbits(24), dqpn=rnd.getrandbits(24),
                       ackreq=rnd.getrandbits(1), solicited=rnd.getrandbits(1),
                       becn=1 if op == 0x81 else 0)
            fr = o.build_frame("10.1.1.48", "10.1.1.15", rnd.getrandbits(24) & 0xFFFF, bth,
                               ext=ext(rnd), payload=payload)
            add(f"rc_{nm}_{pl}", fr, kind="opcode", opcode=op, payload=pl)
    base = o.build_frame("10.1.1.64", "10.1.1.48", 17, dict(opcode=0x0A, psn=99, dqpn=0x42),
                         ext=o.reth_bytes(1, 2, 3), payload=bytes(range(200)))
    add("mask_base", base, kind="mask_base")
    for i in range(16):
        b = bytearray(base)
        for k in (1, 8, 10, 11, 26, 27, 32):
            b[k] = rnd.getrandbits(8)
        b[32] |= rnd.getrandbits(8)
        add(f"mask_variant_{i}", bytes(b), kind="mask_variant")
    for k, what in [(4, "ip_id_hi"), (5, "ip_id_lo"), (6, "ip_flags"), (9, "ip_proto_bit1"),
                    (30, "pkey"), (36, "ackreq_resv7"), (37, "psn"), (40, "reth_va"),
                    (100, "payload"), (len(base) - 5, "last_payload_byte")]:
        b = bytearray(base)
        b[k] ^= 0x02 if what == "ip_proto_bit1" else 0x01
        add(f"sensitivity_{what}", bytes(b), kind="sensitivity")
    # IPv4 with options: masks move with the UDP/BTH offsets
    opt = bytearray(base[:20]) + bytes([1, 1, 1, 0]) + base[20:]
    opt[0] = 0x46
    opt[2:4] = len(opt).to_bytes(2, "big")
    add("ipv4_options_ihl6", bytes(opt), kind="options")
    add("not_ipv4", b"\x60" + base[1:], kind="warning_path")
    add("not_udp", base[:9] + b"\x06" + base[10:], kind="warning_path")

    (HERE / "frames.bin").write_bytes(bytes(blob))
    (HERE / "vectors.json").write_text(json.dumps(
        {"source": "oracle/icrc_oracle.py (zlib.crc32 restatement of src/roce.py:192-223), "
                   "cross-checked with a bitwise CRC seeded 0xDEBB20E3",
         "vectors": vectors}, indent=0) + "\n")
    print(f"{len(vectors)} vectors, {len(blob)} bytes")


if __name__ == "__main__":
    main()
