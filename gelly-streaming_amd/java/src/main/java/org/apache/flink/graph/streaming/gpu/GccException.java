// NOT COMPILED IN THIS IMAGE (no JDK): reference-side bridge, see gelly-streaming_amd/java/README.md
package org.apache.flink.graph.streaming.gpu;

/** A negative status of a libgelly_cc call (include/gelly_cc.h GCC_E_*), with gcc_last_error()'s message. */
public class GccException extends RuntimeException {
    private static final long serialVersionUID = 1L;
    public final int code;

    public GccException(int code, String message) {
        super(message);
        this.code = code;
    }
}
