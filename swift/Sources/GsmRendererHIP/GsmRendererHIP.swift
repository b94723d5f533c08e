// GsmRendererHIP -- the reference's renderer operator surface over the MI355X C ABI.
//
// Mirrors Sources/Renderer/Shared/GaussianRendererProtocol.swift (RenderPrecision :4-7,
// GaussianInput :9-26, CameraParams :28-54, StereoCameraParams :56-66, RendererConfig :195-228,
// StereoRenderTarget :233-239, protocol GaussianRenderer :243-272, RendererError :274-324) and the
// classes GlobalRenderer (Sources/Renderer/GlobalRenderer/GlobalRenderer.swift:72-572) and
// DepthFirstRenderer's side-by-side stereo path (DepthFirstRenderer.swift:205-223).  Metal types
// become HIP ones: MTLBuffer -> HIPBuffer (device pointer + length), MTLTexture -> HIPTexture
// (device pointer + pitch + pixel format), MTLCommandBuffer -> HIPStream (frames are enqueued on
// the stream; the caller synchronises, as it commits a command buffer).  `simd_float4x4` (Apple
// only) becomes Float4x4, four SIMD4<Float> columns with the same column-major memory layout.
//
// UNVERIFIED (no Swift toolchain in the build image); the C call sequence is tested by
// tests/c/abi_sequence.c.
import CGsmAMD

public enum RenderPrecision: Sendable {
    case float32
    case float16
}

/// Device memory: a HIP device pointer and its size in bytes.
public struct HIPBuffer: @unchecked Sendable {
    public let pointer: UnsafeMutableRawPointer
    public let length: Int
    public init(pointer: UnsafeMutableRawPointer, length: Int) {
        self.pointer = pointer
        self.length = length
    }
}

/// The colour formats a target may have (RendererConfig.colorFormat; gsm_color_format).
public enum PixelFormat: UInt32, Sendable {
    case rgba16Float = 0
    case rgba32Float = 1
    case rgba8Unorm = 2
    case rgba8Unorm_srgb = 3
    case bgra8Unorm = 4
    case bgra8Unorm_srgb = 5
    case r16Float = 100  // depth targets

    public var bytesPerPixel: Int {
        switch self {
        case .rgba16Float: 8
        case .rgba32Float: 16
        case .r16Float: 2
        default: 4
        }
    }
}

/// A render target in device memory: `height` rows of `pitch` bytes.
public struct HIPTexture: @unchecked Sendable {
    public let pointer: UnsafeMutableRawPointer
    public let width: Int
    public let height: Int
    public let pitch: Int
    public let pixelFormat: PixelFormat
    public init(pointer: UnsafeMutableRawPointer, width: Int, height: Int, pixelFormat: PixelFormat, pitch: Int? = nil) {
        self.pointer = pointer
        self.width = width
        self.height = height
        self.pixelFormat = pixelFormat
        self.pitch = pitch ?? width * pixelFormat.bytesPerPixel
    }
}

/// The command buffer's role: an ordered HIP stream (nil = the null stream).
public struct HIPStream: @unchecked Sendable {
    public let handle: UnsafeMutableRawPointer?
    public init(handle: UnsafeMutableRawPointer?) { self.handle = handle }
    public static let null = HIPStream(handle: nil)
    public func synchronize() { _ = hipStreamSynchronize(handle) }
}

public struct Float4x4: Sendable {
    public var columns: (SIMD4<Float>, SIMD4<Float>, SIMD4<Float>, SIMD4<Float>)
    public init(columns: (SIMD4<Float>, SIMD4<Float>, SIMD4<Float>, SIMD4<Float>)) { self.columns = columns }
    public static let identity = Float4x4(columns: (SIMD4(1, 0, 0, 0), SIMD4(0, 1, 0, 0), SIMD4(0, 0, 1, 0),
                                                    SIMD4(0, 0, 0, 1)))
    var flat: [Float] {
        [columns.0, columns.1, columns.2, columns.3].flatMap { [$0.x, $0.y, $0.z, $0.w] }
    }
}

public struct GaussianInput: Sendable {
    public let gaussians: HIPBuffer  // PackedWorldGaussian (48 B) or PackedWorldGaussianHalf (32 B)
    public let harmonics: HIPBuffer  // planar SH, float or half
    public let gaussianCount: Int
    public let shComponents: Int
    public init(gaussians: HIPBuffer, harmonics: HIPBuffer, gaussianCount: Int, shComponents: Int) {
        self.gaussians = gaussians
        self.harmonics = harmonics
        self.gaussianCount = gaussianCount
        self.shComponents = shComponents
    }
}

public struct CameraParams: Sendable {
    public let viewMatrix: Float4x4
    public let projectionMatrix: Float4x4
    public let position: SIMD3<Float>
    public let focalX: Float
    public let focalY: Float
    public let near: Float
    public let far: Float
    public init(viewMatrix: Float4x4, projectionMatrix: Float4x4, position: SIMD3<Float>, focalX: Float,
                focalY: Float, near: Float = 0.1, far: Float = 10.0) {
        self.viewMatrix = viewMatrix
        self.projectionMatrix = projectionMatrix
        self.position = position
        self.focalX = focalX
        self.focalY = focalY
        self.near = near
        self.far = far
    }

    var c: gsm_camera_params {
        var cam = gsm_camera_params()
        let v = viewMatrix.flat, p = projectionMatrix.flat
        let pos: [Float] = [position.x, position.y, position.z]
        v.withUnsafeBufferPointer { vb in
            p.withUnsafeBufferPointer { pb in
                pos.withUnsafeBufferPointer { qb in
                    gsm_camera_params_init(&cam, vb.baseAddress, pb.baseAddress, qb.baseAddress, focalX, focalY)
                }
            }
        }
        cam.near_plane = near
        cam.far_plane = far
        return cam
    }
}

public struct StereoCameraParams: Sendable {
    public let leftEye: CameraParams
    public let rightEye: CameraParams
    public init(leftEye: CameraParams, rightEye: CameraParams) {
        self.leftEye = leftEye
        self.rightEye = rightEye
    }
}

public struct RendererConfig: Sendable {
    public enum GaussianColorSpace: UInt32, Sendable {
        case linear = 0
        case srgb = 1
    }

    public let maxGaussians: Int
    public let maxWidth: Int
    public let maxHeight: Int
    public let precision: RenderPrecision
    public let colorFormat: PixelFormat
    public let gaussianColorSpace: GaussianColorSpace
    public let backToFront: Bool

    public init(maxGaussians: Int = 6_000_000, maxWidth: Int = 1920, maxHeight: Int = 1080,
                precision: RenderPrecision = .float16, colorFormat: PixelFormat = .bgra8Unorm_srgb,
                gaussianColorSpace: GaussianColorSpace = .srgb, backToFront: Bool = false) {
        self.maxGaussians = maxGaussians
        self.maxWidth = maxWidth
        self.maxHeight = maxHeight
        self.precision = precision
        self.colorFormat = colorFormat
        self.gaussianColorSpace = gaussianColorSpace
        self.backToFront = backToFront
    }

    var c: gsm_renderer_config {
        var cfg = gsm_renderer_config()
        gsm_renderer_config_default(&cfg)
        cfg.max_gaussians = UInt32(maxGaussians)
        cfg.max_width = UInt32(maxWidth)
        cfg.max_height = UInt32(maxHeight)
        cfg.precision = precision == .float16 ? 1 : 0
        cfg.color_format = colorFormat.rawValue
        cfg.gaussian_color_space = gaussianColorSpace.rawValue
        cfg.back_to_front = backToFront ? 1 : 0
        return cfg
    }
}

/// Stereo targets: side by side only (the reference's foveated Compositor Services drawable has no
/// counterpart off Apple platforms).
public enum StereoRenderTarget: Sendable {
    case sideBySide(colorTexture: HIPTexture, depthTexture: HIPTexture?)
}

public protocol GaussianRenderer: AnyObject {
    var device: Int32 { get }
    var lastGPUTime: Double? { get }

    func render(commandBuffer: HIPStream, colorTexture: HIPTexture, depthTexture: HIPTexture?,
                input: GaussianInput, camera: CameraParams, width: Int, height: Int)

    func renderStereo(commandBuffer: HIPStream, target: StereoRenderTarget, input: GaussianInput,
                      camera: StereoCameraParams, width: Int, height: Int)
}

public enum RendererError: Error, Sendable, Equatable {
    case deviceNotAvailable
    case failedToCreateLibrary
    case failedToCreatePipeline
    case failedToAllocateBuffer
    case failedToAllocateTexture
    case invalidGaussianCount
    case invalidDimensions
    case invalidBufferSize
    case invalidTileCount
    case invalidAssignmentCapacity
    case renderFailed
    case encoderCreationFailed
    case missingRequiredBuffer
    case invalidArgument
    case unsupported

    init?(status: gsm_status) {
        switch status {
        case GSM_OK: return nil
        case GSM_ERR_DEVICE_NOT_AVAILABLE: self = .deviceNotAvailable
        case GSM_ERR_FAILED_TO_CREATE_LIBRARY: self = .failedToCreateLibrary
        case GSM_ERR_FAILED_TO_CREATE_PIPELINE: self = .failedToCreatePipeline
        case GSM_ERR_FAILED_TO_ALLOCATE_BUFFER: self = .failedToAllocateBuffer
        case GSM_ERR_FAILED_TO_ALLOCATE_TEXTURE: self = .failedToAllocateTexture
        case GSM_ERR_INVALID_GAUSSIAN_COUNT: self = .invalidGaussianCount
        case GSM_ERR_INVALID_DIMENSIONS: self = .invalidDimensions
        case GSM_ERR_INVALID_BUFFER_SIZE: self = .invalidBufferSize
        case GSM_ERR_INVALID_TILE_COUNT: self = .invalidTileCount
        case GSM_ERR_INVALID_ASSIGNMENT_CAPACITY: self = .invalidAssignmentCapacity
        case GSM_ERR_RENDER_FAILED: self = .renderFailed
        case GSM_ERR_ENCODER_CREATION_FAILED: self = .encoderCreationFailed
        case GSM_ERR_MISSING_REQUIRED_BUFFER: self = .missingRequiredBuffer
        case GSM_ERR_UNSUPPORTED: self = .unsupported
        case GSM_ERR_PHASE_ORDER: self = .invalidArgument
        default: self = .invalidArgument
        }
    }
}

private func inputStruct(_ input: GaussianInput) -> gsm_gaussian_input {
    gsm_gaussian_input(gaussians: UnsafeRawPointer(input.gaussians.pointer),
                       harmonics: UnsafeRawPointer(input.harmonics.pointer),
                       gaussian_count: UInt32(input.gaussianCount), sh_components: UInt32(input.shComponents))
}

/// GlobalRenderer (GlobalRenderer.swift:72-572) on one HIP device.  Like the reference, `render`
/// does not throw; where the reference silently skips a frame (:295-299) the status is kept in
/// `lastError`.  `renderStereo` is fatalError in the reference's Global path (:240-255): here it
/// sets `lastError = .unsupported`.
public final class GlobalRenderer: GaussianRenderer {
    private var handle: OpaquePointer?
    public let device: Int32
    public private(set) var lastError: RendererError?

    public init(device: Int32 = -1, config: RendererConfig = RendererConfig()) throws {
        var cfg = config.c
        var h: OpaquePointer?
        if let err = RendererError(status: gsm_global_create(&cfg, device, &h)) { throw err }
        handle = h
        self.device = device
    }

    deinit { gsm_global_destroy(handle) }

    public var lastGPUTime: Double? {
        var s = 0.0
        return gsm_global_last_gpu_time(handle, &s) == GSM_OK ? s : nil
    }

    public func render(commandBuffer: HIPStream, colorTexture: HIPTexture, depthTexture: HIPTexture?,
                       input: GaussianInput, camera: CameraParams, width: Int, height: Int) {
        var inp = inputStruct(input)
        var cam = camera.c
        lastError = RendererError(status: gsm_global_render(
            handle, commandBuffer.handle, &inp, &cam, UInt32(width), UInt32(height), colorTexture.pointer,
            colorTexture.pitch, depthTexture?.pointer, depthTexture?.pitch ?? 0))
    }

    public func renderStereo(commandBuffer: HIPStream, target: StereoRenderTarget, input: GaussianInput,
                             camera: StereoCameraParams, width: Int, height: Int) {
        lastError = .unsupported
    }

    /// Config 5 through two Global views (gsm_global_render_stereo_sbs).
    public func renderStereoTwoViews(commandBuffer: HIPStream, target: StereoRenderTarget, input: GaussianInput,
                                     camera: StereoCameraParams, width: Int, height: Int) {
        guard case let .sideBySide(color, depth) = target else { return }
        var inp = inputStruct(input)
        var l = camera.leftEye.c, r = camera.rightEye.c
        lastError = RendererError(status: gsm_global_render_stereo_sbs(
            handle, commandBuffer.handle, &inp, &l, &r, UInt32(width), UInt32(height), color.pointer, color.pitch,
            depth?.pointer, depth?.pitch ?? 0))
    }

    /// debugReadTotalAssignments (GlobalRenderer.swift:196-199).
    public func debugReadTotalAssignments() -> Int { Int(gsm_global_debug_read_total_assignments(handle)) }
}

/// DepthFirstRenderer's side-by-side stereo path (DepthFirstRenderer.swift:205-223).
public final class DepthFirstRenderer: GaussianRenderer {
    private var handle: OpaquePointer?
    public let device: Int32
    public private(set) var lastError: RendererError?

    public init(device: Int32 = -1, config: RendererConfig = RendererConfig()) throws {
        var cfg = config.c
        var h: OpaquePointer?
        if let err = RendererError(status: gsm_depthfirst_create(&cfg, device, &h)) { throw err }
        handle = h
        self.device = device
    }

    deinit { gsm_depthfirst_destroy(handle) }

    public var lastGPUTime: Double? {
        var s = 0.0
        return gsm_depthfirst_last_gpu_time(handle, &s) == GSM_OK ? s : nil
    }

    /// Mono rendering of the DepthFirst renderer is outside this build's scope (DESIGN.md 9).
    public func render(commandBuffer: HIPStream, colorTexture: HIPTexture, depthTexture: HIPTexture?,
                       input: GaussianInput, camera: CameraParams, width: Int, height: Int) {
        lastError = .unsupported
    }

    public func renderStereo(commandBuffer: HIPStream, target: StereoRenderTarget, input: GaussianInput,
                             camera: StereoCameraParams, width: Int, height: Int) {
        guard case let .sideBySide(color, _) = target else { return }
        var inp = inputStruct(input)
        var l = camera.leftEye.c, r = camera.rightEye.c
        lastError = RendererError(status: gsm_depthfirst_render_stereo_sbs(
            handle, commandBuffer.handle, &inp, &l, &r, nil, UInt32(width), UInt32(height), color.pointer,
            color.pitch))
    }
}
