"""CPU oracle for the moseq2-detectron-extract hot path.

TEST INFRASTRUCTURE ONLY.  Only ``tests/``, ``__graft_entry__.smoke()`` and the
``cpu_baseline`` leg of ``bench.py`` may import anything from this package, and
only as the checker / the timed CPU baseline.  The product package
(``moseq2-detectron-extract_amd``) never imports it and fails loudly when its
HIP library is missing instead of falling back to this code.

* ``oracle.frameops``  -- ctypes wrapper over ``frameops.c`` (C restatement of
  the proc/ frame ops, OpenCV semantics restated).
* ``oracle.model_ref`` -- PyTorch-CPU fp32 restatement of the Detectron2
  Mask/Keypoint R-CNN inference path (torchvision ops restated).
"""
