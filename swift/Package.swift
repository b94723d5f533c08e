// swift-tools-version:5.9
// Swift host layer over libgsm_amd.so (SURVEY.md 8(f) row 3): the reference's GaussianRenderer
// operator surface (Sources/Renderer/Shared/GaussianRendererProtocol.swift:243-272) with HIP device
// buffers and streams in place of MTLBuffer / MTLTexture / MTLCommandBuffer.
//
// UNVERIFIED: there is no Swift toolchain in the build image, so this package has never been
// compiled here.  tests/c/abi_sequence.c makes the same C-ABI call sequence as the wrapper below
// and runs in the GPU test suite (tests/test_c_abi.py).
//
// Build: make -C ../gsm-renderer_amd, then
//   swift build -Xlinker -L../gsm-renderer_amd/lib -Xlinker -L/opt/rocm/lib
import PackageDescription

let package = Package(
    name: "GsmRendererHIP",
    products: [
        .library(name: "GsmRendererHIP", targets: ["GsmRendererHIP"]),
    ],
    targets: [
        // the C ABI: include/gsm_renderer.h, gsm_depthfirst.h, gsm_debug.h, gsm_multigpu.h
        .systemLibrary(name: "CGsmAMD", path: "Sources/CGsmAMD"),
        .target(name: "GsmRendererHIP", dependencies: ["CGsmAMD"], path: "Sources/GsmRendererHIP"),
        .testTarget(name: "GsmRendererHIPTests", dependencies: ["GsmRendererHIP"],
                    path: "Tests/GsmRendererHIPTests"),
    ]
)
