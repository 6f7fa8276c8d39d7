"""hipdedisp — MI355X-native replacement for the dedispersion stage of the PALFA
pipeline (pipeline2.0 bin/search.py -> PALFA2_presto_search.search_job -> prepsubband).

Layers:
  _lib           ctypes binding of libhipdedisp.so (include/hipdedisp.h)
  engine         Engine (device context) / Plan (one DDplan pass), PrestoError
  plan           dedisp_plan, hard-coded DDplans, choose_N, DDplan2b restatement
  formats        PSRFITS, .inf, rfifind .mask / .stats, .subNN / .dat
  search_stage   run_pass(): drop-in for PALFA2_presto_search.py:500-529
  prepsubband    command-line shim accepting the reference's prepsubband flags
  synth          synthetic PALFA-shaped beams
  sharding       multi-GPU pass / beam partitioning
"""
from .engine import Engine, ObsParams, Opts, PassParams, Plan, PrestoError, device_count, stats_padvals  # noqa: F401
from .plan import choose_N, dedisp_plan, ddplans_for  # noqa: F401

__version__ = "0.1.0"
