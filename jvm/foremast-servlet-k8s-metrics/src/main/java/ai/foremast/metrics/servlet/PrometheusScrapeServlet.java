package ai.foremast.metrics.servlet;

import io.prometheus.client.exporter.common.TextFormat;

import javax.servlet.ServletConfig;
import javax.servlet.http.HttpServlet;
import javax.servlet.http.HttpServletRequest;
import javax.servlet.http.HttpServletResponse;
import java.io.IOException;
import java.io.Writer;
import java.util.Collections;
import java.util.HashMap;
import java.util.Map;

/**
 * The Prometheus text exposition of the application's {@link ForemastMetrics}
 * registry: map it on {@code /metrics} (the path the foremast ServiceMonitor
 * scrapes) and, for parity with Boot 2 services, {@code /actuator/prometheus}.
 */
public class PrometheusScrapeServlet extends HttpServlet {

    private ForemastMetrics metrics;

    @Override
    public void init(ServletConfig config) {
        Map<String, String> s = new HashMap<>();
        for (String k : Collections.list(config.getInitParameterNames())) {
            s.put(k, config.getInitParameter(k));
        }
        metrics = ForemastMetrics.shared(s);
    }

    @Override
    protected void doGet(HttpServletRequest req, HttpServletResponse resp) throws IOException {
        resp.setStatus(HttpServletResponse.SC_OK);
        resp.setContentType(TextFormat.CONTENT_TYPE_004);
        try (Writer w = resp.getWriter()) {
            w.write(metrics.registry().scrape());
        }
    }
}
