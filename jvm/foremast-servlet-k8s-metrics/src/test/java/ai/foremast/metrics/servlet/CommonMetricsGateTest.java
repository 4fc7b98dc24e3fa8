package ai.foremast.metrics.servlet;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.config.MeterFilterReply;
import org.junit.Test;

import java.io.BufferedReader;
import java.io.InputStreamReader;
import java.nio.charset.StandardCharsets;
import java.util.ArrayList;
import java.util.HashMap;
import java.util.List;
import java.util.Map;

import static org.junit.Assert.assertEquals;
import static org.junit.Assert.fail;

/**
 * Runs gate-vectors.txt (the table tests/test_jvm_starter.py runs through the
 * Python emitter's filter) through {@link CommonMetricsGate}.
 */
public class CommonMetricsGateTest {

    @Test
    public void decisionsMatchTheSharedTable() throws Exception {
        List<String> lines = new ArrayList<>();
        try (BufferedReader r = new BufferedReader(new InputStreamReader(
                getClass().getResourceAsStream("/gate-vectors.txt"), StandardCharsets.UTF_8))) {
            for (String l; (l = r.readLine()) != null; ) {
                l = l.trim();
                if (!l.isEmpty() && !l.startsWith("#")) {
                    lines.add(l);
                }
            }
        }
        lines.add("case end");
        String name = null;
        Map<String, String> settings = new HashMap<>();
        List<String> steps = new ArrayList<>();
        int cases = 0;
        for (String l : lines) {
            if (l.startsWith("case ")) {
                if (name != null) {
                    run(name, settings, steps);
                    cases++;
                }
                name = l.substring(5);
                settings = new HashMap<>();
                steps = new ArrayList<>();
            } else if (l.startsWith("set ")) {
                String kv = l.substring(4);
                int eq = kv.indexOf('=');
                settings.put(kv.substring(0, eq).trim(), kv.substring(eq + 1));
            } else {
                steps.add(l);
            }
        }
        assertEquals(6, cases);
    }

    private static void run(String name, Map<String, String> settings, List<String> steps) {
        CommonMetricsGate gate;
        try {
            gate = new CommonMetricsGate(settings);
        } catch (IllegalArgumentException e) {
            if (!steps.contains("error")) {
                throw e;
            }
            return;
        }
        if (steps.contains("error")) {
            fail(name + ": the settings should not build a gate");
        }
        for (String s : steps) {
            String[] lr = s.split("->");
            String[] w = lr[0].trim().split("\\s+");
            String want = lr[1].trim();
            if ("check".equals(w[0])) {
                List<Tag> tags = new ArrayList<>();
                for (int i = 2; i < w.length; i++) {
                    String[] kv = w[i].split("=", 2);
                    tags.add(Tag.of(kv[0], kv[1]));
                }
                MeterFilterReply got = gate.decide(w[1], tags);
                assertEquals(name + ": " + s, want, got.name());
            } else if ("enable".equals(w[0])) {
                assertEquals(name + ": " + s, Boolean.parseBoolean(want), gate.enableMetric(w[1]));
            } else if ("disable".equals(w[0])) {
                assertEquals(name + ": " + s, Boolean.parseBoolean(want), gate.disableMetric(w[1]));
            } else {
                fail(name + ": unknown step " + s);
            }
        }
    }
}
