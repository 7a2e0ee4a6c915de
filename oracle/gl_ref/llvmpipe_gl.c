/* Run the reference's own vertex + fragment shaders through a real OpenGL
 * driver (Mesa llvmpipe, the software rasteriser the build image ships as
 * swrast_dri.so) and dump the framebuffer.  TEST INFRASTRUCTURE ONLY: it runs
 * in the build container to generate golden images (tests/golden/
 * make_gl_golden.py); nothing under gsviewer_amd/ links, loads or calls it, and
 * it never travels to the GPU box (only the .npz it produces does).
 *
 * No X server, EGL or OSMesa is needed: the harness is its own DRI loader.
 * It dlopens libglapi.so.0 (the GL dispatch) and swrast_dri.so, creates a
 * screen through the DRI swrast interface (GL/internal/dri_interface.h), a
 * GL 4.3 compatibility-profile context, and binds it with no drawable
 * (surfaceless); all rendering goes into a framebuffer object.
 *
 * The frame is drawn as the reference draws it:
 *   - flat() records as SSBO 0, the depth order as SSBO 1
 *     (util.set_storage_buffer_data, renderer_ogl.py:235-242, 263-268);
 *   - the quad VBO/EBO and instanced draw (renderer_ogl.py:144-160, 406-412);
 *   - uniforms through the same glUniform* calls and transposes
 *     (util.py:351-409; set sequence renderer_ogl.py:183-187, 242-318);
 *   - GL_BLEND with SRC_ALPHA / ONE_MINUS_SRC_ALPHA, no face culling
 *     (renderer_ogl.py:178-180); clear to (0,0,0,1) (main.py:197-198).
 * Target: RGBA8 (the viewer's default framebuffer, blending at 8 bits), or
 * RGBA32F with glClampColor(GL_CLAMP_FRAGMENT_COLOR) so each fragment colour
 * is clamped to [0,1] as the unorm target clamps it but the blend is not
 * rounded: the "float" mode of SURVEY Appendix A.5.
 *
 * usage: llvmpipe_gl VERT.glsl FRAG.glsl IN.bin OUT.bin {8|32}
 * IN.bin: struct gl_frame_in (below) then flat float[N*(11+sh_dim)] then
 *         int32 order[N].  OUT.bin: H*W*4 bytes (8) or floats (32), rows
 *         bottom-up as glReadPixels returns them.
 */
#define GL_GLEXT_PROTOTYPES 0
#include <GL/glcorearb.h>
#include <GL/internal/dri_interface.h>
#include <dlfcn.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#ifndef GL_CLAMP_FRAGMENT_COLOR
#define GL_CLAMP_FRAGMENT_COLOR 0x891B
#endif

struct gl_frame_in {
    int32_t w, h, n, sh_dim;
    int32_t render_mod, enable_aabb, enable_obb, pad;
    float view[16];        /* math orientation, row-major (Camera.get_view_matrix) */
    float proj[16];        /* math orientation, row-major */
    float hfovxy_focal[3];
    float cam_pos[3];
    float gaussian_scale_factor, screen_display_scale_factor, dc_factor, extra_factor;
    float color_scale_factors[3];
    float rot_modifier[4]; /* x, y, z, w as util.set_uniform_4f receives them */
    float light_rotation[3];
    float points_center[3];
    float cube_rotation[9]; /* math orientation, row-major */
    float cube_min[3], cube_max[3];
};

static void die(const char *what) {
    fprintf(stderr, "llvmpipe_gl: %s\n", what);
    exit(1);
}

/* ---- the DRI loader side: a surfaceless context needs no drawable callbacks,
 * but the swrast screen wants the loader extension present. */
static void lo_get_drawable_info(__DRIdrawable *d, int *x, int *y, int *w, int *h, void *p) {
    (void)d; (void)p;
    *x = *y = 0; *w = *h = 1;
}
static void lo_put_image(__DRIdrawable *d, int op, int x, int y, int w, int h, char *data, void *p) {
    (void)d; (void)op; (void)x; (void)y; (void)w; (void)h; (void)data; (void)p;
}
static void lo_get_image(__DRIdrawable *d, int x, int y, int w, int h, char *data, void *p) {
    (void)d; (void)x; (void)y; (void)p;
    memset(data, 0, (size_t)w * h * 4);
}
static const __DRIswrastLoaderExtension g_swrast_loader = {
    .base = {__DRI_SWRAST_LOADER, 1},
    .getDrawableInfo = lo_get_drawable_info,
    .putImage = lo_put_image,
    .getImage = lo_get_image,
};
static const __DRIextension *g_loader_exts[] = {&g_swrast_loader.base, NULL};

typedef void *(*get_proc_fn)(const char *);
static get_proc_fn g_get_proc;

#define GLFN(type, name) static type name
GLFN(PFNGLGETERRORPROC, glGetError_);
GLFN(PFNGLGETSTRINGPROC, glGetString_);
GLFN(PFNGLGENFRAMEBUFFERSPROC, glGenFramebuffers_);
GLFN(PFNGLBINDFRAMEBUFFERPROC, glBindFramebuffer_);
GLFN(PFNGLGENRENDERBUFFERSPROC, glGenRenderbuffers_);
GLFN(PFNGLBINDRENDERBUFFERPROC, glBindRenderbuffer_);
GLFN(PFNGLRENDERBUFFERSTORAGEPROC, glRenderbufferStorage_);
GLFN(PFNGLFRAMEBUFFERRENDERBUFFERPROC, glFramebufferRenderbuffer_);
GLFN(PFNGLCHECKFRAMEBUFFERSTATUSPROC, glCheckFramebufferStatus_);
GLFN(PFNGLDRAWBUFFERSPROC, glDrawBuffers_);
GLFN(PFNGLREADBUFFERPROC, glReadBuffer_);
GLFN(PFNGLVIEWPORTPROC, glViewport_);
GLFN(PFNGLCREATESHADERPROC, glCreateShader_);
GLFN(PFNGLSHADERSOURCEPROC, glShaderSource_);
GLFN(PFNGLCOMPILESHADERPROC, glCompileShader_);
GLFN(PFNGLGETSHADERIVPROC, glGetShaderiv_);
GLFN(PFNGLGETSHADERINFOLOGPROC, glGetShaderInfoLog_);
GLFN(PFNGLCREATEPROGRAMPROC, glCreateProgram_);
GLFN(PFNGLATTACHSHADERPROC, glAttachShader_);
GLFN(PFNGLLINKPROGRAMPROC, glLinkProgram_);
GLFN(PFNGLGETPROGRAMIVPROC, glGetProgramiv_);
GLFN(PFNGLGETPROGRAMINFOLOGPROC, glGetProgramInfoLog_);
GLFN(PFNGLUSEPROGRAMPROC, glUseProgram_);
GLFN(PFNGLGENVERTEXARRAYSPROC, glGenVertexArrays_);
GLFN(PFNGLBINDVERTEXARRAYPROC, glBindVertexArray_);
GLFN(PFNGLGENBUFFERSPROC, glGenBuffers_);
GLFN(PFNGLBINDBUFFERPROC, glBindBuffer_);
GLFN(PFNGLBUFFERDATAPROC, glBufferData_);
GLFN(PFNGLBINDBUFFERBASEPROC, glBindBufferBase_);
GLFN(PFNGLGETATTRIBLOCATIONPROC, glGetAttribLocation_);
GLFN(PFNGLVERTEXATTRIBPOINTERPROC, glVertexAttribPointer_);
GLFN(PFNGLENABLEVERTEXATTRIBARRAYPROC, glEnableVertexAttribArray_);
GLFN(PFNGLGETUNIFORMLOCATIONPROC, glGetUniformLocation_);
GLFN(PFNGLUNIFORMMATRIX4FVPROC, glUniformMatrix4fv_);
GLFN(PFNGLUNIFORMMATRIX3FVPROC, glUniformMatrix3fv_);
GLFN(PFNGLUNIFORM1FPROC, glUniform1f_);
GLFN(PFNGLUNIFORM1IPROC, glUniform1i_);
GLFN(PFNGLUNIFORM3FPROC, glUniform3f_);
GLFN(PFNGLUNIFORM4FPROC, glUniform4f_);
GLFN(PFNGLDISABLEPROC, glDisable_);
GLFN(PFNGLENABLEPROC, glEnable_);
GLFN(PFNGLBLENDFUNCPROC, glBlendFunc_);
GLFN(PFNGLCLEARCOLORPROC, glClearColor_);
GLFN(PFNGLCLEARPROC, glClear_);
GLFN(PFNGLDRAWELEMENTSINSTANCEDPROC, glDrawElementsInstanced_);
GLFN(PFNGLFINISHPROC, glFinish_);
GLFN(PFNGLPIXELSTOREIPROC, glPixelStorei_);
GLFN(PFNGLREADPIXELSPROC, glReadPixels_);
GLFN(PFNGLCLAMPCOLORPROC, glClampColor_);

static void *proc(const char *name) {
    void *p = g_get_proc(name);
    if (!p) {
        fprintf(stderr, "llvmpipe_gl: no entry point %s\n", name);
        exit(1);
    }
    return p;
}
#define LOAD(name) name##_ = (__typeof__(name##_))proc(#name)

static void load_gl(void) {
    LOAD(glGetError); LOAD(glGetString); LOAD(glGenFramebuffers); LOAD(glBindFramebuffer);
    LOAD(glGenRenderbuffers); LOAD(glBindRenderbuffer); LOAD(glRenderbufferStorage);
    LOAD(glFramebufferRenderbuffer); LOAD(glCheckFramebufferStatus); LOAD(glDrawBuffers); LOAD(glReadBuffer);
    LOAD(glViewport); LOAD(glCreateShader); LOAD(glShaderSource); LOAD(glCompileShader); LOAD(glGetShaderiv);
    LOAD(glGetShaderInfoLog); LOAD(glCreateProgram); LOAD(glAttachShader); LOAD(glLinkProgram);
    LOAD(glGetProgramiv); LOAD(glGetProgramInfoLog); LOAD(glUseProgram); LOAD(glGenVertexArrays);
    LOAD(glBindVertexArray); LOAD(glGenBuffers); LOAD(glBindBuffer); LOAD(glBufferData); LOAD(glBindBufferBase);
    LOAD(glGetAttribLocation); LOAD(glVertexAttribPointer); LOAD(glEnableVertexAttribArray);
    LOAD(glGetUniformLocation); LOAD(glUniformMatrix4fv); LOAD(glUniformMatrix3fv); LOAD(glUniform1f);
    LOAD(glUniform1i); LOAD(glUniform3f); LOAD(glUniform4f); LOAD(glDisable); LOAD(glEnable); LOAD(glBlendFunc);
    LOAD(glClearColor); LOAD(glClear); LOAD(glDrawElementsInstanced); LOAD(glFinish); LOAD(glPixelStorei);
    LOAD(glReadPixels); LOAD(glClampColor);
}

static void check(const char *where) {
    GLenum e = glGetError_();
    if (e != GL_NO_ERROR) {
        fprintf(stderr, "llvmpipe_gl: GL error 0x%x at %s\n", e, where);
        exit(1);
    }
}

static char *slurp(const char *path, size_t *len) {
    FILE *f = fopen(path, "rb");
    if (!f) {
        fprintf(stderr, "llvmpipe_gl: cannot open %s\n", path);
        exit(1);
    }
    fseek(f, 0, SEEK_END);
    long n = ftell(f);
    fseek(f, 0, SEEK_SET);
    char *b = malloc((size_t)n + 1);
    if (fread(b, 1, (size_t)n, f) != (size_t)n) die("short read");
    b[n] = 0;
    fclose(f);
    if (len) *len = (size_t)n;
    return b;
}

static GLuint compile(GLenum type, const char *src) {
    GLuint s = glCreateShader_(type);
    glShaderSource_(s, 1, &src, NULL);
    glCompileShader_(s);
    GLint ok = 0;
    glGetShaderiv_(s, GL_COMPILE_STATUS, &ok);
    if (!ok) {
        char log[4096];
        glGetShaderInfoLog_(s, sizeof log, NULL, log);
        fprintf(stderr, "llvmpipe_gl: shader compile failed:\n%s\n", log);
        exit(1);
    }
    return s;
}

/* util.set_uniform_mat4 / _mat3 (util.py:351-375): a NumPy matrix M goes up
 * as M.T in C order with transpose=GL_FALSE, i.e. column-major M. */
static void upload_mat4(GLuint prog, const char *name, const float *m) {
    float t[16];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) t[c * 4 + r] = m[r * 4 + c];
    glUniformMatrix4fv_(glGetUniformLocation_(prog, name), 1, GL_FALSE, t);
}
static void upload_mat3(GLuint prog, const char *name, const float *m) {
    float t[9];
    for (int r = 0; r < 3; ++r)
        for (int c = 0; c < 3; ++c) t[c * 3 + r] = m[r * 3 + c];
    glUniformMatrix3fv_(glGetUniformLocation_(prog, name), 1, GL_FALSE, t);
}
static void v3(GLuint prog, const char *name, const float *v) {
    glUniform3f_(glGetUniformLocation_(prog, name), v[0], v[1], v[2]);
}

int main(int argc, char **argv) {
    if (argc != 6) die("usage: llvmpipe_gl VERT FRAG IN.bin OUT.bin {8|32}");
    const int bits = atoi(argv[5]);
    if (bits != 8 && bits != 32) die("target must be 8 or 32");

    size_t in_len = 0;
    char *in = slurp(argv[3], &in_len);
    struct gl_frame_in U;
    if (in_len < sizeof U) die("input too short");
    memcpy(&U, in, sizeof U);
    const size_t rec = 11 + (size_t)U.sh_dim;
    const size_t flat_bytes = (size_t)U.n * rec * 4, order_bytes = (size_t)U.n * 4;
    if (in_len != sizeof U + flat_bytes + order_bytes) die("input size does not match its header");
    const float *flat = (const float *)(in + sizeof U);
    const int32_t *order = (const int32_t *)(in + sizeof U + flat_bytes);

    /* ---- DRI: dispatch library first (global, so the driver binds to it). */
    void *glapi = dlopen("libglapi.so.0", RTLD_NOW | RTLD_GLOBAL);
    if (!glapi) die(dlerror());
    g_get_proc = (get_proc_fn)dlsym(glapi, "_glapi_get_proc_address");
    if (!g_get_proc) die("_glapi_get_proc_address missing");
    const char *drv_path = getenv("LLVMPIPE_DRI_PATH");
    if (!drv_path) drv_path = "/usr/lib/x86_64-linux-gnu/dri/swrast_dri.so";
    void *drv = dlopen(drv_path, RTLD_NOW | RTLD_GLOBAL);
    if (!drv) die(dlerror());
    typedef const __DRIextension **(*get_ext_fn)(void);
    get_ext_fn get_ext = (get_ext_fn)dlsym(drv, "__driDriverGetExtensions_swrast");
    if (!get_ext) die("__driDriverGetExtensions_swrast missing");
    const __DRIextension **drv_exts = get_ext();
    const __DRIcoreExtension *core = NULL;
    const __DRIswrastExtension *sw = NULL;
    for (int i = 0; drv_exts[i]; ++i) {
        if (!strcmp(drv_exts[i]->name, __DRI_CORE)) core = (const __DRIcoreExtension *)drv_exts[i];
        if (!strcmp(drv_exts[i]->name, __DRI_SWRAST)) sw = (const __DRIswrastExtension *)drv_exts[i];
    }
    if (!core || !sw) die("driver lacks DRI_Core / DRI_SWRast");
    if (sw->base.version < 4) die("DRI_SWRast older than version 4 (no createNewScreen2)");
    const __DRIconfig **configs = NULL;
    __DRIscreen *screen = sw->createNewScreen2(0, g_loader_exts, drv_exts, &configs, NULL);
    if (!screen || !configs || !configs[0]) die("createNewScreen2 failed");
    const uint32_t attribs[] = {
        __DRI_CTX_ATTRIB_MAJOR_VERSION, 4,
        __DRI_CTX_ATTRIB_MINOR_VERSION, 3,
    };
    unsigned err = 0;
    /* compatibility profile: glClampColor(GL_CLAMP_FRAGMENT_COLOR) is not in core */
    __DRIcontext *ctx = sw->createContextAttribs(screen, __DRI_API_OPENGL, configs[0], NULL, 2, attribs, &err, NULL);
    if (!ctx) {
        fprintf(stderr, "llvmpipe_gl: createContextAttribs failed, error %u\n", err);
        return 1;
    }
    if (!core->bindContext(ctx, NULL, NULL)) die("bindContext (surfaceless) failed");
    load_gl();
    fprintf(stderr, "llvmpipe_gl: %s | %s\n", (const char *)glGetString_(GL_RENDERER),
            (const char *)glGetString_(GL_VERSION));

    /* ---- render target */
    const int W = U.w, H = U.h;
    GLuint fbo, rb;
    glGenFramebuffers_(1, &fbo);
    glBindFramebuffer_(GL_FRAMEBUFFER, fbo);
    glGenRenderbuffers_(1, &rb);
    glBindRenderbuffer_(GL_RENDERBUFFER, rb);
    glRenderbufferStorage_(GL_RENDERBUFFER, bits == 8 ? GL_RGBA8 : GL_RGBA32F, W, H);
    glFramebufferRenderbuffer_(GL_FRAMEBUFFER, GL_COLOR_ATTACHMENT0, GL_RENDERBUFFER, rb);
    if (glCheckFramebufferStatus_(GL_FRAMEBUFFER) != GL_FRAMEBUFFER_COMPLETE) die("framebuffer incomplete");
    const GLenum db = GL_COLOR_ATTACHMENT0;
    glDrawBuffers_(1, &db);
    glReadBuffer_(GL_COLOR_ATTACHMENT0);
    if (bits == 32) glClampColor_(GL_CLAMP_FRAGMENT_COLOR, GL_TRUE);
    glViewport_(0, 0, W, H);
    check("framebuffer");

    /* ---- program (util.load_shaders, util.py:220-230) */
    char *vs = slurp(argv[1], NULL), *fs = slurp(argv[2], NULL);
    GLuint prog = glCreateProgram_();
    glAttachShader_(prog, compile(GL_VERTEX_SHADER, vs));
    glAttachShader_(prog, compile(GL_FRAGMENT_SHADER, fs));
    glLinkProgram_(prog);
    GLint linked = 0;
    glGetProgramiv_(prog, GL_LINK_STATUS, &linked);
    if (!linked) {
        char log[4096];
        glGetProgramInfoLog_(prog, sizeof log, NULL, log);
        fprintf(stderr, "llvmpipe_gl: link failed:\n%s\n", log);
        return 1;
    }
    glUseProgram_(prog);

    /* ---- quad geometry (renderer_ogl.py:144-160) */
    static const float quad_v[8] = {-1, 1, 1, 1, 1, -1, -1, -1};
    static const uint32_t quad_f[6] = {0, 1, 2, 0, 2, 3};
    GLuint vao, vbo, ebo, ssbo[2];
    glGenVertexArrays_(1, &vao);
    glBindVertexArray_(vao);
    glGenBuffers_(1, &vbo);
    glBindBuffer_(GL_ARRAY_BUFFER, vbo);
    glBufferData_(GL_ARRAY_BUFFER, sizeof quad_v, quad_v, GL_STATIC_DRAW);
    GLint pos = glGetAttribLocation_(prog, "position");
    if (pos < 0) die("no attribute 'position'");
    glVertexAttribPointer_((GLuint)pos, 2, GL_FLOAT, GL_FALSE, 0, NULL);
    glEnableVertexAttribArray_((GLuint)pos);
    glGenBuffers_(1, &ebo);
    glBindBuffer_(GL_ELEMENT_ARRAY_BUFFER, ebo);
    glBufferData_(GL_ELEMENT_ARRAY_BUFFER, sizeof quad_f, quad_f, GL_STATIC_DRAW);
    check("quad");

    /* ---- SSBOs (util.set_storage_buffer_data, util.py:306-321) */
    glGenBuffers_(2, ssbo);
    glBindBuffer_(GL_SHADER_STORAGE_BUFFER, ssbo[0]);
    glBufferData_(GL_SHADER_STORAGE_BUFFER, (GLsizeiptr)(flat_bytes ? flat_bytes : 4), flat, GL_STATIC_DRAW);
    glBindBufferBase_(GL_SHADER_STORAGE_BUFFER, 0, ssbo[0]);
    glBindBuffer_(GL_SHADER_STORAGE_BUFFER, ssbo[1]);
    glBufferData_(GL_SHADER_STORAGE_BUFFER, (GLsizeiptr)(order_bytes ? order_bytes : 4), order, GL_STATIC_DRAW);
    glBindBufferBase_(GL_SHADER_STORAGE_BUFFER, 1, ssbo[1]);
    glBindBuffer_(GL_SHADER_STORAGE_BUFFER, 0);
    check("ssbo");

    /* ---- uniforms (every one the shaders declare; GL zero-initialises the rest) */
    upload_mat4(prog, "view_matrix", U.view);
    upload_mat4(prog, "projection_matrix", U.proj);
    v3(prog, "hfovxy_focal", U.hfovxy_focal);
    v3(prog, "cam_pos", U.cam_pos);
    glUniform1i_(glGetUniformLocation_(prog, "sh_dim"), U.sh_dim);
    glUniform1f_(glGetUniformLocation_(prog, "gaussian_scale_factor"), U.gaussian_scale_factor);
    glUniform1f_(glGetUniformLocation_(prog, "screen_display_scale_factor"), U.screen_display_scale_factor);
    glUniform1f_(glGetUniformLocation_(prog, "dc_factor"), U.dc_factor);
    glUniform1f_(glGetUniformLocation_(prog, "extra_factor"), U.extra_factor);
    v3(prog, "color_scale_factors", U.color_scale_factors);
    glUniform1i_(glGetUniformLocation_(prog, "render_mod"), U.render_mod);
    glUniform4f_(glGetUniformLocation_(prog, "rot_modifier"), U.rot_modifier[0], U.rot_modifier[1],
                 U.rot_modifier[2], U.rot_modifier[3]);
    v3(prog, "light_rotation", U.light_rotation);
    v3(prog, "points_center", U.points_center);
    glUniform1i_(glGetUniformLocation_(prog, "enable_aabb"), U.enable_aabb);
    glUniform1i_(glGetUniformLocation_(prog, "enable_obb"), U.enable_obb);
    upload_mat3(prog, "cube_rotation", U.cube_rotation);
    v3(prog, "cubeMin", U.cube_min);
    v3(prog, "cubeMax", U.cube_max);
    check("uniforms");

    /* ---- GL state (renderer_ogl.py:178-180) and the frame (main.py:197-198, renderer_ogl.py:406-412) */
    glDisable_(GL_CULL_FACE);
    glEnable_(GL_BLEND);
    glBlendFunc_(GL_SRC_ALPHA, GL_ONE_MINUS_SRC_ALPHA);
    glClearColor_(0.f, 0.f, 0.f, 1.0f);
    glClear_(GL_COLOR_BUFFER_BIT);
    if (U.n > 0) glDrawElementsInstanced_(GL_TRIANGLES, 6, GL_UNSIGNED_INT, NULL, U.n);
    glFinish_();
    check("draw");

    const size_t px = (size_t)W * H * 4;
    void *out = malloc(bits == 8 ? px : px * 4);
    glPixelStorei_(GL_PACK_ALIGNMENT, 1);
    glReadPixels_(0, 0, W, H, GL_RGBA, bits == 8 ? GL_UNSIGNED_BYTE : GL_FLOAT, out);
    check("readpixels");
    FILE *f = fopen(argv[4], "wb");
    if (!f) die("cannot write output");
    fwrite(out, 1, bits == 8 ? px : px * 4, f);
    fclose(f);
    core->unbindContext(ctx);
    core->destroyContext(ctx);
    core->destroyScreen(screen);
    return 0;
}
