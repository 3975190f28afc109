package io.vproxy.vpcsum;

import java.io.IOException;
import java.lang.foreign.FunctionDescriptor;
import java.lang.foreign.Linker;
import java.lang.foreign.MemorySegment;
import java.lang.foreign.SymbolLookup;
import java.lang.foreign.ValueLayout;
import java.lang.invoke.MethodHandle;
import java.util.Optional;

/**
 * The library check that must work before anything else of libvpcsum is touched.
 *
 * {@link VPCsum} resolves its PNI downcalls in its static initialiser, as the generated PNI
 * classes do (PosixNative.java:729-744): initialising it without the library loaded fails with an
 * ExceptionInInitializerError.  This class holds no such handle: {@link #requireAbi} resolves
 * vpcsum_abi_version on first use and turns a missing library or a different ABI into an
 * IOException, so {@link GpuCsumBatch} can check before it initialises {@link VPCsum}.
 *
 * Not compiled in this repository (the build image has no JDK); see INTEGRATION.md.
 */
final class VPCsumLib {
    private VPCsumLib() {
    }

    private static volatile MethodHandle abiVersionMH;

    /** vpcsum_abi_version() of the loaded library; IOException when it is not loaded. */
    static int abiVersion() throws IOException {
        MethodHandle mh = abiVersionMH;
        if (mh == null) {
            Optional<MemorySegment> sym = SymbolLookup.loaderLookup().find("vpcsum_abi_version");
            if (sym.isEmpty()) {
                throw new IOException("libvpcsum is not loaded (vpcsum_abi_version not found): load it with " +
                                      "Utils.loadDynamicLibrary(\"vpcsum\") before creating a GpuCsumBatch");
            }
            mh = Linker.nativeLinker().downcallHandle(sym.get(), FunctionDescriptor.of(ValueLayout.JAVA_INT));
            abiVersionMH = mh;
        }
        try {
            return (int) mh.invokeExact();
        } catch (Throwable t) {
            throw new IOException("vpcsum_abi_version failed", t);
        }
    }

    /** IOException unless the loaded library speaks ABI {@code expected} (VPCsum.ABI_VERSION). */
    static void requireAbi(int expected) throws IOException {
        int v = abiVersion();
        if (v != expected) {
            throw new IOException("libvpcsum ABI " + v + ", binding expects " + expected);
        }
    }
}
