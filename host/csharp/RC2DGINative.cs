// RC2DGINative.cs -- P/Invoke binding of librc2dgi.so (include/rc2dgi.h) for the reference's
// C# host (RC2DGI.cs).  Drop this file next to RC2DGI.cs and apply the patch shown in
// INTEGRATION.md: DoRC2DGI() (RC2DGI.cs:267-406) becomes one native call, the uniform
// globals keep their names, and the debug thumbnails (RC2DGI.cs:156-163) are refreshed
// from the native render textures.
//
// Not compiled in this repository (no .NET SDK in the build image); the C ABI it binds is
// exercised by tests/ through the same entry points.
using System;
using System.Runtime.InteropServices;
using Raylib_cs;

static unsafe class RC2DGINative
{
    const string Lib = "rc2dgi"; // librc2dgi.so / rc2dgi.dll on the loader path

    public const int OK = 0;
    public enum RT { Color = 0, Emissive = 1, Jump1 = 2, Jump2 = 3, Dist = 4, GI1 = 5, GI2 = 6, Temp = 7, Blur = 8, FinalGI = 9 }
    public enum Format { RGBA8 = 0, RGBA32F = 1 }
    public enum Storage { F32 = 0, RGBA8Compat = 1, F16 = 2 }  // RGBA8Compat: the shipped app's RGBA8 textures, byte-exact

    [StructLayout(LayoutKind.Sequential)]
    public struct Config
    {
        public int ScreenWidth, ScreenHeight, CascadeCount;
        public float RenderScale, RayRange;
        public int Storage, Device;
        public int Flags;              // 1 = Linux merge fallback (Merge.fs not found, RC2DGI.cs:62)
        public int R0, R1, R2, R3;     // reserved, zero
    }

    [DllImport(Lib)] public static extern int rc2dgi_create(ref Config cfg, out IntPtr ctx);
    [DllImport(Lib)] public static extern int rc2dgi_destroy(IntPtr ctx);
    [DllImport(Lib)] public static extern int rc2dgi_set_uniform(IntPtr ctx, [MarshalAs(UnmanagedType.LPUTF8Str)] string name, float* v, int n);
    [DllImport(Lib)] public static extern int rc2dgi_set_uniform_i(IntPtr ctx, [MarshalAs(UnmanagedType.LPUTF8Str)] string name, int v);
    [DllImport(Lib)] public static extern int rc2dgi_upload(IntPtr ctx, int which, void* host, int pitchBytes, int format);
    [DllImport(Lib)] public static extern int rc2dgi_do(IntPtr ctx);
    [DllImport(Lib)] public static extern int rc2dgi_sync(IntPtr ctx);
    [DllImport(Lib)] public static extern int rc2dgi_download(IntPtr ctx, int which, void* host, int pitchBytes, int format);
    [DllImport(Lib)] public static extern int rc2dgi_query(IntPtr ctx, out int cw, out int ch, out int jfaSteps, out int finalGi);
    [DllImport(Lib)] public static extern IntPtr rc2dgi_last_error(IntPtr ctx);

    // rc2dgi_prim: DrawRectangleRec (Kind 0) / DrawCircleV (Kind 1, W = radius), raylib screen coordinates
    [StructLayout(LayoutKind.Sequential)]
    public struct Prim
    {
        public int Kind;
        public float X, Y, W, H;
        public byte R, G, B, A;
    }
    [DllImport(Lib)] public static extern int rc2dgi_paint(IntPtr ctx, int which, byte* clearRgba, Prim* prims, int n);

    static IntPtr ctx;
    static byte[] scratch = Array.Empty<byte>();

    static void Check(int rc, string what)
    {
        if (rc != OK)
            throw new InvalidOperationException($"{what}: rc2dgi error {rc}: {Marshal.PtrToStringUTF8(rc2dgi_last_error(ctx))}");
    }

    // RC2DGI.cs:65-98 (knobs + render-texture set)
    public static void Init(int screenWidth, int screenHeight, int cascadeCount, float renderScale, float rayRange)
    {
        var cfg = new Config { ScreenWidth = screenWidth, ScreenHeight = screenHeight, CascadeCount = cascadeCount,
                               RenderScale = renderScale, RayRange = rayRange };
        Check(rc2dgi_create(ref cfg, out ctx), "rc2dgi_create");
    }

    public static void Shutdown() { if (ctx != IntPtr.Zero) rc2dgi_destroy(ctx); ctx = IntPtr.Zero; }

    // SetGIShaderValues (RC2DGI.cs:408-433) + the blur radius (RC2DGI.cs:374): same names
    public static void SetUniform(string name, float v) => Check(rc2dgi_set_uniform(ctx, name, &v, 1), name);
    public static void SetUniform(string name, System.Numerics.Vector3 v)
    {
        float* p = stackalloc float[3] { v.X, v.Y, v.Z };
        Check(rc2dgi_set_uniform(ctx, name, p, 3), name);
    }

    // painted colorRT / emissiveRT -> device (RGBA8 in GL row order, as rlReadTexturePixels returns it)
    public static void Upload(RT which, RenderTexture2D rt)
    {
        Image img = Raylib.LoadImageFromTexture(rt.Texture);
        try { Check(rc2dgi_upload(ctx, (int)which, img.Data, rt.Texture.Width * 4, (int)Format.RGBA8), "upload"); }
        finally { Raylib.UnloadImage(img); }
    }

    // device render texture -> the raylib texture that displays it (debug views / final blit)
    public static void Download(RT which, RenderTexture2D rt)
    {
        int n = rt.Texture.Width * rt.Texture.Height * 4;
        if (scratch.Length < n) scratch = new byte[n];
        fixed (byte* p = scratch)
        {
            Check(rc2dgi_download(ctx, (int)which, p, rt.Texture.Width * 4, (int)Format.RGBA8), "download");
            Raylib.UpdateTexture(rt.Texture, p);
        }
    }

    public static Prim Rect(Rectangle r, Color c) => new Prim { Kind = 0, X = r.X, Y = r.Y, W = r.Width, H = r.Height, R = c.R, G = c.G, B = c.B, A = c.A };
    public static Prim Circle(System.Numerics.Vector2 p, float radius, Color c) => new Prim { Kind = 1, X = p.X, Y = p.Y, W = radius, R = c.R, G = c.G, B = c.B, A = c.A };

    // BeginTextureMode(rt); ClearBackground(clear); draw prims; EndTextureMode -- on the GPU
    // (RenderScene / RedrawSceneToRTs, RC2DGI.cs:224-264, 528-545)
    public static void Paint(RT which, Color? clear, System.Collections.Generic.List<Prim> prims)
    {
        Prim[] a = prims.ToArray();
        byte* cl = stackalloc byte[4];
        if (clear is Color c) { cl[0] = c.R; cl[1] = c.G; cl[2] = c.B; cl[3] = c.A; }
        fixed (Prim* p = a)
            Check(rc2dgi_paint(ctx, (int)which, clear.HasValue ? cl : null, p, a.Length), "paint");
    }

    // DoRC2DGI() (RC2DGI.cs:267-406)
    public static void DoRC2DGI() => Check(rc2dgi_do(ctx), "rc2dgi_do");
}
