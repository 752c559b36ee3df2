/* refcl.c -- TEST INFRASTRUCTURE ONLY: a minimal OpenCL host used to run the
 * reference's own kernels (Kernels/Raytracing.cl, compiled from its sources by
 * oracle/Makefile into oracle/_ref/raytracing_gfx950.co, plus the KAT wrapper
 * kat.cl) on the ROCm OpenCL runtime of the GPU box.  It replaces nothing in
 * the product; it plays the role pyopencl plays in KernelLauncher.py (absent
 * from this image): program from binary, buffers, image, enqueue, read back.
 *
 * Exposed to Python (oracle/refcl.py) through ctypes.
 */
#define CL_TARGET_OPENCL_VERSION 200
#include <CL/cl.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#define MAX_KERNELS 32
#define MAX_ARGS 32

static cl_context g_ctx;
static cl_device_id g_dev;
static cl_command_queue g_q;
static cl_program g_prog;
static cl_kernel g_k[MAX_KERNELS];
static int g_nk;
static char g_err[4096];

typedef struct {
    cl_mem mem;
    void* host;
    size_t bytes;
    int readback;
} arg_t;
static arg_t g_args[MAX_KERNELS][MAX_ARGS];

static int fail(const char* what, cl_int e) {
    snprintf(g_err, sizeof g_err, "%s failed (cl error %d)", what, (int)e);
    return -1;
}

const char* refcl_error(void) { return g_err; }

int refcl_open(const char* co_path) {
    cl_int e;
    cl_platform_id plats[8];
    cl_uint np = 0;
    if ((e = clGetPlatformIDs(8, plats, &np)) != CL_SUCCESS || np == 0) return fail("clGetPlatformIDs", e);
    int found = 0;
    for (cl_uint p = 0; p < np && !found; ++p) {
        cl_uint nd = 0;
        if (clGetDeviceIDs(plats[p], CL_DEVICE_TYPE_GPU, 1, &g_dev, &nd) == CL_SUCCESS && nd > 0) found = 1;
    }
    if (!found) return fail("clGetDeviceIDs(GPU)", -1);
    g_ctx = clCreateContext(NULL, 1, &g_dev, NULL, NULL, &e);
    if (e != CL_SUCCESS) return fail("clCreateContext", e);
    g_q = clCreateCommandQueue(g_ctx, g_dev, CL_QUEUE_PROFILING_ENABLE, &e);
    if (e != CL_SUCCESS) return fail("clCreateCommandQueue", e);
    FILE* f = fopen(co_path, "rb");
    if (!f) { snprintf(g_err, sizeof g_err, "cannot open %s", co_path); return -1; }
    fseek(f, 0, SEEK_END);
    size_t len = (size_t)ftell(f);
    fseek(f, 0, SEEK_SET);
    unsigned char* bin = (unsigned char*)malloc(len);
    if (fread(bin, 1, len, f) != len) { fclose(f); free(bin); return fail("fread", -1); }
    fclose(f);
    cl_int bst;
    const unsigned char* bins[1] = {bin};
    g_prog = clCreateProgramWithBinary(g_ctx, 1, &g_dev, &len, bins, &bst, &e);
    free(bin);
    if (e != CL_SUCCESS) return fail("clCreateProgramWithBinary", e);
    e = clBuildProgram(g_prog, 1, &g_dev, "", NULL, NULL);
    if (e != CL_SUCCESS) {
        size_t l = 0;
        clGetProgramBuildInfo(g_prog, g_dev, CL_PROGRAM_BUILD_LOG, sizeof g_err - 64, g_err + 64, &l);
        snprintf(g_err, 64, "clBuildProgram failed (%d): ", (int)e);
        return -1;
    }
    g_nk = 0;
    return 0;
}

int refcl_device_name(char* out, int n) {
    return clGetDeviceInfo(g_dev, CL_DEVICE_NAME, (size_t)n, out, NULL) == CL_SUCCESS ? 0 : -1;
}

int refcl_kernel(const char* name) {
    if (g_nk >= MAX_KERNELS) return fail("too many kernels", -1);
    cl_int e;
    g_k[g_nk] = clCreateKernel(g_prog, name, &e);
    if (e != CL_SUCCESS) return fail(name, e);
    memset(g_args[g_nk], 0, sizeof g_args[g_nk]);
    return g_nk++;
}

int refcl_arg_buf(int k, int idx, void* host, size_t bytes, int readback) {
    cl_int e;
    if (bytes == 0) bytes = 4;
    cl_mem_flags fl = readback ? CL_MEM_READ_WRITE : CL_MEM_READ_ONLY;
    if (host) fl |= CL_MEM_COPY_HOST_PTR;
    cl_mem m = clCreateBuffer(g_ctx, fl, bytes, host, &e);
    if (e != CL_SUCCESS) return fail("clCreateBuffer", e);
    g_args[k][idx].mem = m;
    g_args[k][idx].host = host;
    g_args[k][idx].bytes = bytes;
    g_args[k][idx].readback = readback;
    if ((e = clSetKernelArg(g_k[k], (cl_uint)idx, sizeof(cl_mem), &m)) != CL_SUCCESS) return fail("clSetKernelArg(buf)", e);
    return 0;
}

int refcl_arg_scalar(int k, int idx, const void* val, size_t size) {
    cl_int e = clSetKernelArg(g_k[k], (cl_uint)idx, size, val);
    return e == CL_SUCCESS ? 0 : fail("clSetKernelArg(scalar)", e);
}

int refcl_arg_image(int k, int idx, const uint8_t* rgba, int w, int h) {
    cl_int e;
    cl_image_format fmt = {CL_RGBA, CL_UNORM_INT8};
    cl_image_desc desc;
    memset(&desc, 0, sizeof desc);
    desc.image_type = CL_MEM_OBJECT_IMAGE2D;
    desc.image_width = (size_t)w;
    desc.image_height = (size_t)h;
    cl_mem m = clCreateImage(g_ctx, CL_MEM_READ_ONLY | CL_MEM_COPY_HOST_PTR, &fmt, &desc, (void*)rgba, &e);
    if (e != CL_SUCCESS) return fail("clCreateImage", e);
    g_args[k][idx].mem = m;
    g_args[k][idx].readback = 0;
    if ((e = clSetKernelArg(g_k[k], (cl_uint)idx, sizeof(cl_mem), &m)) != CL_SUCCESS) return fail("clSetKernelArg(img)", e);
    return 0;
}

/* Enqueue over `global` work-items (local size left to the runtime, as
 * KernelLauncher.py:76 does), wait, read back, release the arguments. */
int refcl_run(int k, size_t global, double* kernel_ms) {
    cl_int e;
    cl_event ev;
    e = clEnqueueNDRangeKernel(g_q, g_k[k], 1, NULL, &global, NULL, 0, NULL, &ev);
    if (e != CL_SUCCESS) return fail("clEnqueueNDRangeKernel", e);
    if ((e = clWaitForEvents(1, &ev)) != CL_SUCCESS) return fail("clWaitForEvents", e);
    if (kernel_ms) {
        cl_ulong t0 = 0, t1 = 0;
        clGetEventProfilingInfo(ev, CL_PROFILING_COMMAND_START, sizeof t0, &t0, NULL);
        clGetEventProfilingInfo(ev, CL_PROFILING_COMMAND_END, sizeof t1, &t1, NULL);
        *kernel_ms = (double)(t1 - t0) * 1e-6;
    }
    clReleaseEvent(ev);
    for (int i = 0; i < MAX_ARGS; ++i) {
        arg_t* a = &g_args[k][i];
        if (a->mem && a->readback && a->host) {
            e = clEnqueueReadBuffer(g_q, a->mem, CL_TRUE, 0, a->bytes, a->host, 0, NULL, NULL);
            if (e != CL_SUCCESS) return fail("clEnqueueReadBuffer", e);
        }
    }
    for (int i = 0; i < MAX_ARGS; ++i) {
        if (g_args[k][i].mem) clReleaseMemObject(g_args[k][i].mem);
        g_args[k][i].mem = NULL;
    }
    return 0;
}

void refcl_close(void) {
    for (int i = 0; i < g_nk; ++i) clReleaseKernel(g_k[i]);
    g_nk = 0;
    if (g_prog) clReleaseProgram(g_prog);
    if (g_q) clReleaseCommandQueue(g_q);
    if (g_ctx) clReleaseContext(g_ctx);
    g_prog = NULL; g_q = NULL; g_ctx = NULL;
}
