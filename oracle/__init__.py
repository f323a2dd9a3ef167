"""ORACLE — TEST INFRASTRUCTURE ONLY.

CPU restatement of the reference's detection hot path (torch_models/detect.py:62-105 and the
torchvision eval path it calls at detect.py:78), plus a restatement of the ORIE consumer
(reward.py:16-69, lib/metrics.py, lib/data.py:11-84).

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may import
anything under ``oracle/`` — as the checker, never as the thing measured or shipped.  The product
package (``edgeml-object-detection_amd/``) never imports it.

Pinning:
  * output formatting (detect.py:79-105) and the ORIE consumer are pinned byte-for-byte by golden
    fixtures generated from the reference itself (tests/golden/make_golden.py);
  * the model arithmetic lives in torchvision, which is absent from this container and unpinned by
    the reference.  Its restatement here is pinned by the analytic known answers the
    survey derived (parameter counts 3,440,060 / 5,198,540 / 43,712,278, anchor counts 3,234 and
    159,882) — the model arithmetic itself is otherwise "parity unpinned" against torchvision.
"""
