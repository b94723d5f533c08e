// UNVERIFIED (no Swift toolchain in the build image).  The same sequence runs from C in
// tests/c/abi_sequence.c (tests/test_c_abi.py, GPU suite).
import CGsmAMD
import XCTest

@testable import GsmRendererHIP

final class GlobalRendererTests: XCTestCase {
    // GlobalRenderer.init guard (GlobalRenderer.swift:111-113)
    func testTooManyGaussiansThrows() {
        XCTAssertThrowsError(try GlobalRenderer(config: RendererConfig(maxGaussians: 30_000_001))) { err in
            XCTAssertEqual(err as? RendererError, .invalidGaussianCount)
        }
    }

    // an empty frame: cleared target (0, 0, 0, 1) and no assignments (GlobalShaders.metal:140-154)
    func testEmptyFrameClears() throws {
        let w = 64, h = 32
        let r = try GlobalRenderer(device: 0, config: RendererConfig(maxGaussians: 16, maxWidth: w, maxHeight: h,
                                                                     colorFormat: .rgba16Float))
        var color: UnsafeMutableRawPointer?
        var scratch: UnsafeMutableRawPointer?
        XCTAssertEqual(hipMalloc(&color, w * h * 8), 0)
        XCTAssertEqual(hipMalloc(&scratch, 64), 0)
        defer { _ = hipFree(color); _ = hipFree(scratch) }
        let buf = HIPBuffer(pointer: scratch!, length: 64)
        let input = GaussianInput(gaussians: buf, harmonics: buf, gaussianCount: 0, shComponents: 1)
        let cam = CameraParams(viewMatrix: .identity, projectionMatrix: .identity, position: .zero, focalX: 1, focalY: 1)
        r.render(commandBuffer: .null, colorTexture: HIPTexture(pointer: color!, width: w, height: h,
                                                                pixelFormat: .rgba16Float),
                 depthTexture: nil, input: input, camera: cam, width: w, height: h)
        HIPStream.null.synchronize()
        XCTAssertNil(r.lastError)
        XCTAssertEqual(r.debugReadTotalAssignments(), 0)
        var host = [UInt16](repeating: 0, count: w * h * 4)
        _ = host.withUnsafeMutableBytes { hipMemcpy($0.baseAddress, color, w * h * 8, 2) }
        XCTAssertEqual(host[3], 0x3C00)  // alpha 1.0h
        // renderStereo is fatalError in the reference's Global path: here an error, not a trap
        r.renderStereo(commandBuffer: .null,
                       target: .sideBySide(colorTexture: HIPTexture(pointer: color!, width: w, height: h,
                                                                    pixelFormat: .rgba16Float), depthTexture: nil),
                       input: input, camera: StereoCameraParams(leftEye: cam, rightEye: cam), width: w / 2, height: h)
        XCTAssertEqual(r.lastError, .unsupported)
    }
}
