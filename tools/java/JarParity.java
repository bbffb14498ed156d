/*
 * JarParity — one-command boundary parity check of the committed CDC fixtures against the real
 * rabinwindow jar, for a host that HAS a JDK and org.opendedupe:rabinwindow:1.0.2 (pom.xml:92-96).
 * This container has neither (SURVEY.md 8(c)), so the file is source only; nothing here runs it.
 *
 *   javac -cp rabinwindow-1.0.2.jar -d /tmp/jp tools/java/JarParity.java
 *   java  -cp rabinwindow-1.0.2.jar:/tmp/jp JarParity tests/golden/cdc.json [--emit tests/golden/jar_cdc.json]
 *
 * What it does, per fixture of tests/golden/cdc.json (made by tests/golden/make_golden.py):
 *   1. rebuilds the input bytes from the fixture's generator spec (the counter-based SplitMix64
 *      stream of oracle/cdc_ref.c cdc_ref_synth, zeros, a fill byte, a ramp, a zero hole) and checks
 *      them against the fixture's input_sha256;
 *   2. chunks them exactly as VariableSha256HashEngine.getChunks does (VariableSha256HashEngine.java:
 *      41-52,71-86): new EnhancedFingerFactory(Polynomial.createFromLong(poly), window,
 *      BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR, minLen, maxLen).getChunkFingerprints(data, visitor),
 *      SHA-256 / first 20 bytes / MD5 of every visited chunk (Guava's Hashing.sha256()/md5() wrap the
 *      JDK MessageDigest, so MessageDigest is used here and Guava is not needed);
 *   3. diffs (start, len, digest) against the fixture and prints MATCH or the first difference.
 * The jar's detector is fixed (DEFAULT_BOUNDARY_DETECTOR), so only fixtures whose predicate knobs
 * equal the jar's can match: the summary names the fixtures that match and prints the detector
 * object's class and fields (reflection), i.e. which sdfs_cdc_params predicate form and constants
 * (SDFS_CDC_PRED_MASK / SDFS_CDC_PRED_DIV, include/sdfs_cdc.h) reproduce the jar.  --emit writes the
 * jar's own chunk lists for every fixture input as JSON; committed as tests/golden/jar_cdc.json,
 * tests/test_gpu_parity.py::test_jar_fixtures_bit_exact then pins the GPU path to the jar itself.
 *
 * --sdfs additionally runs the stock org.opendedup.hashing.VariableSha256HashEngine (by reflection,
 * with HashFunctionPool.minLen / maxLen / bytesPerWindow set first) when the SDFS jar and its
 * logging dependencies are on the class path, and checks that it equals step 2.
 */
import java.io.FileOutputStream;
import java.io.IOException;
import java.io.OutputStreamWriter;
import java.io.Writer;
import java.lang.reflect.Field;
import java.lang.reflect.Modifier;
import java.nio.charset.StandardCharsets;
import java.nio.file.Files;
import java.nio.file.Paths;
import java.security.MessageDigest;
import java.util.ArrayList;
import java.util.LinkedHashMap;
import java.util.List;
import java.util.Map;

import org.rabinfingerprint.handprint.BoundaryDetectors;
import org.rabinfingerprint.handprint.EnhancedFingerFactory;
import org.rabinfingerprint.handprint.EnhancedFingerFactory.EnhancedChunkVisitor;
import org.rabinfingerprint.polynomial.Polynomial;

public final class JarParity {

    // ---------------------------------------------------------------- input generators
    static long splitmix64(long x) {
        long z = x + 0x9E3779B97F4A7C15L;
        z = (z ^ (z >>> 30)) * 0xBF58476D1CE4E5B9L;
        z = (z ^ (z >>> 27)) * 0x94D049BB133111EBL;
        return z ^ (z >>> 31);
    }

    /** byte o of stream s = little-endian byte (o % 8) of splitmix64(key + o / 8),
     *  key = splitmix64(seed ^ (s * 0xD1B54A32D192ED03)) — oracle/cdc_ref.c cdc_ref_synth. */
    static byte[] synth(long seed, long stream, long offset, int n) {
        long key = splitmix64(seed ^ (stream * 0xD1B54A32D192ED03L));
        byte[] out = new byte[n];
        for (int i = 0; i < n; i++) {
            long o = offset + i;
            long w = splitmix64(key + (o >>> 3));
            out[i] = (byte) (w >>> (8 * (int) (o & 7)));
        }
        return out;
    }

    static long num(Map<String, Object> m, String k, long dflt) {
        Object v = m.get(k);
        return v == null ? dflt : ((Number) v).longValue();
    }

    @SuppressWarnings("unchecked")
    static byte[] makeInput(Map<String, Object> spec, long defaultSeed) {
        String kind = (String) spec.get("kind");
        int n = (int) num(spec, "len", 0);
        switch (kind) {
            case "synth":
                return synth(num(spec, "seed", defaultSeed), num(spec, "stream", 0), num(spec, "offset", 0), n);
            case "zeros":
                return new byte[n];
            case "fill": {
                byte[] b = new byte[n];
                java.util.Arrays.fill(b, (byte) num(spec, "byte", 0));
                return b;
            }
            case "ramp": {
                byte[] b = new byte[n];
                for (int i = 0; i < n; i++) b[i] = (byte) (i & 0xFF);
                return b;
            }
            case "splice": {
                byte[] b = synth(defaultSeed, num(spec, "stream", 0), 0, n);
                int h0 = (int) num(spec, "hole_start", 0), hl = (int) num(spec, "hole_len", 0);
                for (int i = h0; i < Math.min(n, h0 + hl); i++) b[i] = 0;
                return b;
            }
            default:
                throw new IllegalArgumentException("unknown input kind " + kind);
        }
    }

    // ---------------------------------------------------------------- the reference loop
    static final class Chunk {
        final long start, len;
        final byte[] digest;
        Chunk(long start, long len, byte[] digest) { this.start = start; this.len = len; this.digest = digest; }
    }

    static byte[] digest(int algo, byte[] chunk) throws Exception {
        MessageDigest md = MessageDigest.getInstance(algo == 2 ? "MD5" : "SHA-256");
        byte[] h = md.digest(chunk);
        if (algo == 1) return java.util.Arrays.copyOf(h, 20);  // HASH160, VariableSha256HashEngine.java:60-65
        return h;
    }

    /** VariableSha256HashEngine.getChunks (:71-86) with the jar's factory and default detector. */
    static List<Chunk> jarChunks(byte[] data, long poly, long window, int minLen, int maxLen, final int algo) {
        EnhancedFingerFactory ff = new EnhancedFingerFactory(Polynomial.createFromLong(poly), window,
                BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR, minLen, maxLen);
        final List<Chunk> out = new ArrayList<>();
        final Exception[] err = new Exception[1];
        ff.getChunkFingerprints(data, new EnhancedChunkVisitor() {
            public void visit(long fingerprint, long chunkStart, long chunkEnd, byte[] chunk) {
                try {
                    out.add(new Chunk(chunkStart, chunkEnd - chunkStart, digest(algo, chunk)));
                } catch (Exception e) {
                    err[0] = e;
                }
            }
        });
        if (err[0] != null) throw new RuntimeException(err[0]);
        return out;
    }

    /** The stock engine, by reflection (needs the SDFS jar + its logging on the class path). */
    @SuppressWarnings("unchecked")
    static List<Chunk> sdfsChunks(byte[] data, long window, int minLen, int maxLen, int algo) throws Exception {
        Class<?> pool = Class.forName("org.opendedup.hashing.HashFunctionPool");
        pool.getField("minLen").setInt(null, minLen);
        pool.getField("maxLen").setInt(null, maxLen);
        pool.getField("bytesPerWindow").setLong(null, window);
        Class<?> eng = Class.forName("org.opendedup.hashing.VariableSha256HashEngine");
        Class<?> ht = Class.forName("org.opendedup.hashing.VariableSha256HashEngine$HASHTYPE");
        Object hash = Enum.valueOf((Class<Enum>) ht, algo == 1 ? "HASH160" : "HASH256");
        Object e = eng.getConstructor(ht).newInstance(hash);
        List<?> fingers = (List<?>) eng.getMethod("getChunks", byte[].class, String.class).invoke(e, data, "jar-parity");
        List<Chunk> out = new ArrayList<>();
        for (Object f : fingers) {
            Class<?> fc = f.getClass();
            out.add(new Chunk(fc.getField("start").getInt(f), fc.getField("len").getInt(f),
                    (byte[]) fc.getField("hash").get(f)));
        }
        return out;
    }

    // ---------------------------------------------------------------- compare / report
    static String hex(byte[] b) {
        StringBuilder s = new StringBuilder();
        for (byte x : b) s.append(String.format("%02x", x & 0xFF));
        return s.toString();
    }

    @SuppressWarnings("unchecked")
    static String diff(List<Chunk> got, Map<String, Object> fx) {
        List<Object> st = (List<Object>) fx.get("starts"), ln = (List<Object>) fx.get("lens"),
                dg = (List<Object>) fx.get("digests");
        int n = Math.min(got.size(), st.size());
        for (int i = 0; i < n; i++) {
            Chunk c = got.get(i);
            long es = ((Number) st.get(i)).longValue(), el = ((Number) ln.get(i)).longValue();
            if (c.start != es || c.len != el)
                return "chunk " + i + ": jar (" + c.start + "," + c.len + ") fixture (" + es + "," + el + ")";
            if (!hex(c.digest).equals(dg.get(i))) return "chunk " + i + ": digest differs";
        }
        if (got.size() != st.size()) return "jar " + got.size() + " chunks, fixture " + st.size();
        return null;
    }

    static void describeDetector() {
        Object d = BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR;
        System.out.println("DEFAULT_BOUNDARY_DETECTOR = " + d.getClass().getName());
        for (Class<?> c = d.getClass(); c != null && c != Object.class; c = c.getSuperclass())
            for (Field f : c.getDeclaredFields()) {
                if (Modifier.isStatic(f.getModifiers())) continue;
                try {
                    f.setAccessible(true);
                    Object v = f.get(d);
                    String s = v instanceof Long ? String.format("%d (0x%x)", v, v) : String.valueOf(v);
                    System.out.println("  " + f.getName() + " = " + s);
                } catch (Exception e) {
                    System.out.println("  " + f.getName() + " = <" + e + ">");
                }
            }
        System.out.println("  -> set sdfs.hip.boundary to mask:<mask>:<value> (a bitmask detector) or div:<divisor>:<target>"
                + " (a divisor detector), and min_cmp to whichever of the matching fixtures' min_cmp (0: n > minLen,"
                + " 1: n >= minLen) agrees");
    }

    @SuppressWarnings("unchecked")
    public static void main(String[] args) throws Exception {
        if (args.length < 1) {
            System.err.println("usage: JarParity tests/golden/cdc.json [--emit out.json] [--sdfs]");
            System.exit(2);
        }
        String emit = null;
        boolean sdfs = false;
        for (int i = 1; i < args.length; i++) {
            if (args[i].equals("--emit") && i + 1 < args.length) emit = args[++i];
            else if (args[i].equals("--sdfs")) sdfs = true;
        }
        Map<String, Object> root = (Map<String, Object>) new Json(new String(Files.readAllBytes(Paths.get(args[0])),
                StandardCharsets.UTF_8)).value();
        long seed = num(root, "seed", 0x5DF50001L);
        describeDetector();
        List<String> matched = new ArrayList<>();
        List<Map<String, Object>> emitted = new ArrayList<>();
        int bad = 0;
        for (Object o : (List<Object>) root.get("fixtures")) {
            Map<String, Object> fx = (Map<String, Object>) o;
            Map<String, Object> p = (Map<String, Object>) fx.get("params");
            byte[] data = makeInput((Map<String, Object>) fx.get("input"), seed);
            String sha = hex(MessageDigest.getInstance("SHA-256").digest(data));
            if (!sha.equals(fx.get("input_sha256"))) {
                System.out.println(fx.get("name") + ": INPUT MISMATCH (generator restatement wrong)");
                bad++;
                continue;
            }
            long poly = num(p, "poly", 10923124345206883L), window = num(p, "window", 48);
            int minLen = (int) num(p, "min_len", 4095), maxLen = (int) num(p, "max_len", 32768);
            int algo = (int) num(p, "hash_algo", 0);
            List<Chunk> got = jarChunks(data, poly, window, minLen, maxLen, algo);
            if (sdfs) {
                String d2 = diffChunks(got, sdfsChunks(data, window, minLen, maxLen, algo));
                if (d2 != null) {
                    System.out.println(fx.get("name") + ": stock VariableSha256HashEngine differs from the factory loop: " + d2);
                    bad++;
                }
            }
            String d = diff(got, fx);
            System.out.println(String.format("%-22s %s  params %s", fx.get("name"), d == null ? "MATCH" : "differs: " + d, p));
            if (d == null) matched.add((String) fx.get("name"));
            if (emit != null) {
                Map<String, Object> e = new LinkedHashMap<>();
                e.put("name", fx.get("name"));
                e.put("input", fx.get("input"));
                e.put("input_sha256", sha);
                Map<String, Object> jp = new LinkedHashMap<>();
                jp.put("poly", poly); jp.put("window", window); jp.put("min_len", (long) minLen);
                jp.put("max_len", (long) maxLen); jp.put("hash_algo", (long) algo);
                e.put("jar_params", jp);
                List<Object> s = new ArrayList<>(), l = new ArrayList<>(), g = new ArrayList<>();
                for (Chunk c : got) { s.add(c.start); l.add(c.len); g.add(hex(c.digest)); }
                e.put("starts", s); e.put("lens", l); e.put("digests", g);
                emitted.add(e);
            }
        }
        System.out.println("matching fixtures: " + matched);
        if (emit != null) {
            Map<String, Object> out = new LinkedHashMap<>();
            out.put("note", "chunk lists of the rabinwindow jar itself (tools/java/JarParity.java --emit)");
            out.put("detector", BoundaryDetectors.DEFAULT_BOUNDARY_DETECTOR.getClass().getName());
            out.put("seed", seed);
            out.put("fixtures", emitted);
            try (Writer w = new OutputStreamWriter(new FileOutputStream(emit), StandardCharsets.UTF_8)) {
                Json.write(w, out);
            }
            System.out.println("wrote " + emit);
        }
        System.exit(bad == 0 ? 0 : 1);
    }

    static String diffChunks(List<Chunk> a, List<Chunk> b) {
        if (a.size() != b.size()) return a.size() + " vs " + b.size() + " chunks";
        for (int i = 0; i < a.size(); i++)
            if (a.get(i).start != b.get(i).start || a.get(i).len != b.get(i).len
                    || !java.util.Arrays.equals(a.get(i).digest, b.get(i).digest))
                return "chunk " + i;
        return null;
    }

    // ---------------------------------------------------------------- minimal JSON (no dependencies)
    static final class Json {
        private final String s;
        private int i;
        Json(String s) { this.s = s; }

        Object value() {
            ws();
            char c = s.charAt(i);
            if (c == '{') return object();
            if (c == '[') return array();
            if (c == '"') return string();
            if (s.startsWith("true", i)) { i += 4; return Boolean.TRUE; }
            if (s.startsWith("false", i)) { i += 5; return Boolean.FALSE; }
            if (s.startsWith("null", i)) { i += 4; return null; }
            return number();
        }

        private void ws() { while (i < s.length() && Character.isWhitespace(s.charAt(i))) i++; }

        private Map<String, Object> object() {
            Map<String, Object> m = new LinkedHashMap<>();
            i++;
            ws();
            if (s.charAt(i) == '}') { i++; return m; }
            for (;;) {
                ws();
                String k = string();
                ws();
                i++;  // ':'
                m.put(k, value());
                ws();
                if (s.charAt(i++) == '}') return m;  // else ','
            }
        }

        private List<Object> array() {
            List<Object> a = new ArrayList<>();
            i++;
            ws();
            if (s.charAt(i) == ']') { i++; return a; }
            for (;;) {
                a.add(value());
                ws();
                if (s.charAt(i++) == ']') return a;  // else ','
            }
        }

        private String string() {
            StringBuilder b = new StringBuilder();
            i++;  // opening quote
            for (;;) {
                char c = s.charAt(i++);
                if (c == '"') return b.toString();
                if (c == '\\') {
                    char e = s.charAt(i++);
                    if (e == 'u') { b.append((char) Integer.parseInt(s.substring(i, i + 4), 16)); i += 4; }
                    else b.append(e == 'n' ? '\n' : e == 't' ? '\t' : e == 'r' ? '\r' : e == 'b' ? '\b' : e == 'f' ? '\f' : e);
                } else {
                    b.append(c);
                }
            }
        }

        private Number number() {
            int j = i;
            while (i < s.length() && "+-0123456789.eE".indexOf(s.charAt(i)) >= 0) i++;
            String t = s.substring(j, i);
            if (t.indexOf('.') >= 0 || t.indexOf('e') >= 0 || t.indexOf('E') >= 0) return Double.parseDouble(t);
            return new java.math.BigInteger(t).longValue();  // u64 values above 2^63 keep their bits
        }

        @SuppressWarnings("unchecked")
        static void write(Writer w, Object v) throws IOException {
            if (v == null) w.write("null");
            else if (v instanceof String) w.write("\"" + ((String) v).replace("\\", "\\\\").replace("\"", "\\\"") + "\"");
            else if (v instanceof Number || v instanceof Boolean) w.write(String.valueOf(v));
            else if (v instanceof Map) {
                w.write("{");
                boolean first = true;
                for (Map.Entry<String, Object> e : ((Map<String, Object>) v).entrySet()) {
                    if (!first) w.write(",");
                    first = false;
                    write(w, e.getKey());
                    w.write(":");
                    write(w, e.getValue());
                }
                w.write("}");
            } else if (v instanceof List) {
                w.write("[");
                boolean first = true;
                for (Object o : (List<Object>) v) {
                    if (!first) w.write(",");
                    first = false;
                    write(w, o);
                }
                w.write("]");
            } else {
                throw new IOException("cannot write " + v.getClass());
            }
        }
    }
}
