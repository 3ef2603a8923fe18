"""fluere_amd -- MI355X-native drop-in for fluere's `offline` pcap->flow hot path
(and its `live` mode on batched capture, fluere_amd.live).

The compute path is the in-tree HIP library (fluere_amd/libfluere_gpu.so,
C ABI in include/fluere_gpu.h); this package is the host-side mirror of the
reference's offline-mode seams.  See DESIGN.md.
"""
from . import dist, live  # noqa: F401
from ._lib import FluereError, available  # noqa: F401
from .offline import (Args, Files, FlowContext, FluereRecord, Parameters, fluere_exporter,  # noqa: F401
                      fluereflow_fileparse, format_csv, synth_cfg, synth_device, synth_device_batches,
                      synth_pcap)

__all__ = ["Args", "Files", "Parameters", "FlowContext", "FluereRecord", "FluereError", "available",
           "fluere_exporter", "fluereflow_fileparse", "format_csv", "synth_cfg", "synth_device",
           "synth_device_batches", "synth_pcap"]
