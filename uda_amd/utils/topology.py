"""Device discovery and shuffle planning for one node (netlev device/link discovery).

The reference discovers InfiniBand devices and sizes queue pairs (src/DataNet/RDMAComm.cc:320-358);
here the node is a set of MI355X GPUs joined point-to-point by xGMI (7 links of ~153 GB/s per GPU).
`topology()` reports what HIP sees; `shuffle_plan()` turns it into the all-to-all schedule the engine
uses: the rotating peer order (every step each GPU sends on a different link) and a round size that
keeps each per-peer message large enough to run the links at speed.
"""
from __future__ import annotations

from .._native import native

XGMI = 2  # HSA_AMD_LINK_INFO_TYPE_XGMI
XGMI_LINK_GBPS = 153.0
PCIE_GEN5_X16_GBPS = 63.0


def topology() -> dict:
    """{'devices': n, 'props': [...], 'links': [{'src','dst','p2p','link_type','hops','perf_rank'}]}"""
    return native().device_topology()


def peer_order(rank: int, world: int) -> list[tuple[int, int]]:
    """(send_to, recv_from) per step; step k pairs rank with rank±k so all links carry one message."""
    return [((rank + k) % world, (rank - k) % world) for k in range(1, world)]


def shuffle_plan(world: int, bytes_per_gpu: int, hbm_bytes: int = 288 << 30,
                 min_msg_bytes: int = 64 << 20) -> dict:
    """Rounds for the key-range shuffle: a round must fit the HBM staging budget (send + receive +
    merge workspace ~ 4x the round) and each peer message should stay >= min_msg_bytes so RCCL runs
    the xGMI links near line rate."""
    staging = hbm_bytes // 8
    rounds_mem = max(1, -(-4 * bytes_per_gpu // max(1, 4 * staging)))
    per_peer = bytes_per_gpu / max(1, world)
    rounds_msg = max(1, int(per_peer // min_msg_bytes)) if world > 1 else 1
    rounds = max(rounds_mem, min(16, rounds_msg))
    return {
        "world": world,
        "rounds": rounds,
        "bytes_per_round": bytes_per_gpu // rounds,
        "peer_msg_bytes": int(per_peer // rounds),
        "xgmi_egress_gbps": XGMI_LINK_GBPS * min(7, max(0, world - 1)),
        "d2h_bound_gbps": PCIE_GEN5_X16_GBPS,
    }


def describe() -> str:
    t = topology()
    lines = [f"{t['devices']} HIP device(s)"]
    for i, p in enumerate(t["props"]):
        lines.append(f"  gpu{i}: {p['name']} {p['arch']} {p['cus']} CUs, {p['hbm_bytes'] / 2**30:.0f} GiB")
    xgmi = sum(1 for l in t["links"] if l["link_type"] == XGMI)
    if t["links"]:
        lines.append(f"  {xgmi}/{len(t['links'])} device pairs over xGMI")
    return "\n".join(lines)


if __name__ == "__main__":
    print(describe())
