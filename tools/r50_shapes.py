"""The R50 conv shapes the tile tools time (name, cin, cout, k, stride, hin, residual, wlimbs)."""
SHAPES = [  # name, cin, cout, k, stride, hin, residual, wlimbs
    ("c1_256_64_56", 256, 64, 1, 1, 56, False, 1),
    # the first block of each stage: conv1 on the stage input (once per stage)
    ("c1f_64_64_56", 64, 64, 1, 1, 56, False, 1),
    ("c1f_256_128_56", 256, 128, 1, 1, 56, False, 1),
    ("c1f_512_256_28", 512, 256, 1, 1, 28, False, 1),
    ("c1f_1024_512_14", 1024, 512, 1, 1, 14, False, 1),
    ("c2_64_64_56", 64, 64, 3, 1, 56, False, 1),
    ("c3_64_256_56r", 64, 256, 1, 1, 56, True, 1),
    ("c2_128_128_28", 128, 128, 3, 1, 28, False, 1),
    ("c2_128_128_56s2", 128, 128, 3, 2, 56, False, 1),
    ("c1_512_128_28", 512, 128, 1, 1, 28, False, 1),
    ("c3_128_512_28r", 128, 512, 1, 1, 28, True, 1),
    ("c2_256_256_14", 256, 256, 3, 1, 14, False, 1),
    ("c1_1024_256_14", 1024, 256, 1, 1, 14, False, 1),
    ("c3_256_1024_14r", 256, 1024, 1, 1, 14, True, 1),
    ("c2_512_512_7", 512, 512, 3, 1, 7, False, 1),
    # BasicBlock conv2 (R18 / R34): 3x3 + the identity as limb planes, then ReLU
    ("c2r_64_64_56", 64, 64, 3, 1, 56, True, 1),
    ("c2r_128_128_28", 128, 128, 3, 1, 28, True, 1),
    ("c2r_256_256_14", 256, 256, 3, 1, 14, True, 1),
    ("c2r_512_512_7", 512, 512, 3, 1, 7, True, 1),
    ("c1_2048_512_7", 2048, 512, 1, 1, 7, False, 1),
    ("ds_1024_2048_14s2", 1024, 2048, 1, 2, 14, False, 3),
    ("ds_512_1024_28s2", 512, 1024, 1, 2, 28, False, 3),
    ("ds_256_512_56s2", 256, 512, 1, 2, 56, False, 3),
    ("ds_64_256_56", 64, 256, 1, 1, 56, False, 3),
    # the strided downsamples on an input already subsampled by 2 (same outputs, stride 1)
    # the BasicBlock nets' (R18 / R34) strided downsamples
    ("ds18_64_128_56s2", 64, 128, 1, 2, 56, False, 3),
    ("ds18_128_256_28s2", 128, 256, 1, 2, 28, False, 3),
    ("ds18_256_512_14s2", 256, 512, 1, 2, 14, False, 3),
    ("dsq_1024_2048_7s1", 1024, 2048, 1, 1, 7, False, 3),
    ("dsq_512_1024_14s1", 512, 1024, 1, 1, 14, False, 3),
    ("dsq_256_512_28s1", 256, 512, 1, 1, 28, False, 3),
]
