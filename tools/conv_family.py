"""The synthesis conv kernel family as profiles name it (shared by the rocprof / PMC summary tools): every kernel
smc_conv_gemm_f32 / smc_conv3x3_wino_f32 / smc_conv3x3_wino4_f32 launch for the synthesis (TAG 0).  The IR-SE50 executor's launches of
the same GEMM kernels carry TAG 1 (a trailing ", 1>" template argument) and are not part of it."""

FAMILY = ("conv_gemm_lds_kernel", "conv_gemm_kernel", "conv_row_kernel", "convt_gemm_kernel", "convt_lds_kernel",
          "conv_gemm_x3_kernel", "convt_x3_kernel", "wino_kernel", "wino4_kernel")


def is_family(name):
    return any(f in name for f in FAMILY) and ", 1>(" not in name


def is_wino(name):
    return "wino_kernel" in name or "wino4_kernel" in name
