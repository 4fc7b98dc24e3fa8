package ai.foremast.metrics.boot1;

import ai.foremast.metrics.servlet.ForemastMetricsListener;
import ai.foremast.metrics.servlet.HttpRequestsFilter;
import ai.foremast.metrics.servlet.MetricsControlServlet;
import ai.foremast.metrics.servlet.PrometheusScrapeServlet;
import org.springframework.boot.autoconfigure.condition.ConditionalOnProperty;
import org.springframework.boot.autoconfigure.condition.ConditionalOnWebApplication;
import org.springframework.boot.bind.RelaxedPropertyResolver;
import org.springframework.boot.web.servlet.FilterRegistrationBean;
import org.springframework.boot.web.servlet.ServletListenerRegistrationBean;
import org.springframework.boot.web.servlet.ServletRegistrationBean;
import org.springframework.context.annotation.Bean;
import org.springframework.context.annotation.Configuration;
import org.springframework.core.Ordered;
import org.springframework.core.env.Environment;

import javax.servlet.Filter;
import javax.servlet.FilterChain;
import javax.servlet.FilterConfig;
import javax.servlet.ServletException;
import javax.servlet.ServletRequest;
import javax.servlet.ServletResponse;
import javax.servlet.http.HttpServletResponse;
import java.io.IOException;
import java.util.HashMap;
import java.util.Map;

/**
 * Spring Boot 1.5 auto-configuration of the servlet metrics module (the
 * reference 1.x starter, foremast-spring-boot-1x-k8s-metrics-starter/.../
 * K8sMetricsAutoConfiguration.java): the request filter on every path, the
 * scrape servlet on /prometheus and /actuator/prometheus, /metrics answered
 * with a redirect there (the reference's K8sMetricsFilter: Kubernetes scrapes
 * /metrics by default), runtime enable / disable on /k8s-metrics/*, and the
 * Tomcat session binder.  Every {@code k8s.metrics.*} property is handed to the
 * module as its setting of the same (camel-case) name, e.g.
 * {@code k8s.metrics.common-metrics-whitelist} -> {@code commonMetricsWhitelist},
 * {@code k8s.metrics.caller-default} -> {@code callerDefault};
 * {@code management.metrics.enable.*} become the gate's {@code enable.*}.
 * {@code k8s.metrics.enabled=false} turns it all off.
 */
@Configuration
@ConditionalOnWebApplication
@ConditionalOnProperty(prefix = "k8s.metrics", name = "enabled", havingValue = "true", matchIfMissing = true)
public class Boot1MetricsAutoConfiguration {

    static final String[] SETTINGS = {"app", "callerHeader", "callerDefault", "initializeForStatuses", "jvmMetrics",
        "tomcatMetrics", "enableCommonMetricsFilter", "enableCommonMetricsFilterAction", "commonMetricsWhitelist",
        "commonMetricsBlacklist", "commonMetricsPrefix", "commonMetricsTagRules"};

    /** k8s.metrics.* (relaxed names) -> the servlet module's settings. */
    static Map<String, String> settings(Environment env) {
        Map<String, String> out = new HashMap<>();
        RelaxedPropertyResolver k8s = new RelaxedPropertyResolver(env, "k8s.metrics.");
        for (String name : SETTINGS) {
            String v = k8s.getProperty(name);
            if (v != null) {
                out.put(name, v);
            }
        }
        String app = env.getProperty("info.app.name");
        if (app != null && !out.containsKey("app")) {
            out.put("app", app);                 // the reference's app:ENV.APP_NAME|info.app.name
        }
        RelaxedPropertyResolver enable = new RelaxedPropertyResolver(env, "management.metrics.enable.");
        for (Map.Entry<String, Object> e : enable.getSubProperties("").entrySet()) {
            out.put("enable." + e.getKey(), String.valueOf(e.getValue()));
        }
        return out;
    }

    private static <T extends org.springframework.boot.web.servlet.RegistrationBean> T params(T bean, Environment env) {
        bean.setInitParameters(settings(env));
        return bean;
    }

    @Bean
    public FilterRegistrationBean foremastRequestsFilter(Environment env) {
        FilterRegistrationBean b = params(new FilterRegistrationBean(new HttpRequestsFilter()), env);
        b.addUrlPatterns("/*");
        b.setOrder(Ordered.HIGHEST_PRECEDENCE + 10);
        return b;
    }

    @Bean
    public ServletRegistrationBean foremastPrometheusServlet(Environment env) {
        return params(new ServletRegistrationBean(new PrometheusScrapeServlet(), "/prometheus",
                "/actuator/prometheus"), env);
    }

    @Bean
    public ServletRegistrationBean foremastMetricsControl(Environment env) {
        return params(new ServletRegistrationBean(new MetricsControlServlet(), "/k8s-metrics/*"), env);
    }

    @Bean
    public ServletListenerRegistrationBean<ForemastMetricsListener> foremastTomcatBinder() {
        return new ServletListenerRegistrationBean<>(new ForemastMetricsListener());
    }

    /** /metrics -> /prometheus (Kubernetes scrapes /metrics by default). */
    @Bean
    @ConditionalOnProperty(prefix = "k8s.metrics", name = "redirect-metrics", havingValue = "true",
            matchIfMissing = true)
    public FilterRegistrationBean foremastMetricsRedirect() {
        FilterRegistrationBean b = new FilterRegistrationBean(new Filter() {
            public void init(FilterConfig c) {
            }

            public void doFilter(ServletRequest req, ServletResponse res, FilterChain chain)
                    throws IOException, ServletException {
                if (res instanceof HttpServletResponse) {
                    ((HttpServletResponse) res).sendRedirect("/prometheus");
                } else {
                    chain.doFilter(req, res);
                }
            }

            public void destroy() {
            }
        });
        b.addUrlPatterns("/metrics");
        b.setOrder(Ordered.HIGHEST_PRECEDENCE);
        return b;
    }
}
