"""vproxy_amd -- MI355X-native (gfx950 HIP) batched Internet checksum engine for vproxy's vswitch.

The product is ``libvpcsum.so`` (C-ABI: ``include/vpcsum.h``); this package builds it in-tree
(:mod:`vproxy_amd.build`), binds it (:mod:`vproxy_amd.vpcsum`) and mirrors the vswitch egress
seam that calls it (:mod:`vproxy_amd.vswitch`).
"""
__all__ = ["build", "vpcsum", "vswitch", "shard"]
