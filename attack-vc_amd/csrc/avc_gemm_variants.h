// conv_gemm tile variants: (index, precision, WM, WN, WGM, WGN, KC, name)
// tile = 32*WM*WGM x 32*WN*WGN, 64*WGM*WGN threads; included with
// AVC_GEMM_VARIANT defined (instantiation in avc_gemm.hip, dispatch in avc_api.hip).
AVC_GEMM_VARIANT(0, PREC_F32, 2, 1, 2, 4, 32, "conv_gemm_f32<128x128,w8,k32>")
AVC_GEMM_VARIANT(1, PREC_F32, 2, 2, 2, 2, 32, "conv_gemm_f32<128x128,w4,k32>")
AVC_GEMM_VARIANT(2, PREC_F32, 2, 1, 2, 2, 32, "conv_gemm_f32<128x64,w4,k32>")
AVC_GEMM_VARIANT(3, PREC_F32, 1, 1, 2, 2, 32, "conv_gemm_f32<64x64,w4,k32>")
AVC_GEMM_VARIANT(4, PREC_F32, 1, 1, 2, 4, 32, "conv_gemm_f32<64x128,w8,k32>")
AVC_GEMM_VARIANT(5, PREC_BF16, 2, 1, 2, 4, 64, "conv_gemm_bf16<128x128,w8,k64>")
AVC_GEMM_VARIANT(6, PREC_BF16, 2, 2, 2, 2, 32, "conv_gemm_bf16<128x128,w4,k32>")
AVC_GEMM_VARIANT(7, PREC_BF16, 2, 1, 2, 2, 32, "conv_gemm_bf16<128x64,w4,k32>")
AVC_GEMM_VARIANT(8, PREC_BF16, 1, 1, 2, 2, 32, "conv_gemm_bf16<64x64,w4,k32>")
AVC_GEMM_VARIANT(9, PREC_BF16, 1, 1, 2, 4, 64, "conv_gemm_bf16<64x128,w8,k64>")
